// K5 / K6 — GATConv edge softmax + attention-weighted aggregation, forward and backward.
//
// Replaces PyG 2.5.3 GATConv (constructed at src/models/gnn.py:64-67, called at :72,75):
//   alpha_src = (xh * att_src).sum(-1); alpha_dst = (xh * att_dst).sum(-1)
//   remove_self_loops; add_self_loops                      -> GNN_LOOPS_REPLACE plan
//   edge_update: e = leaky_relu(alpha_src[j] + alpha_dst[i], 0.2)
//   utils.softmax: exp(e - scatter_max(e.detach())[i]) / (scatter_sum(exp)[i] + 1e-16)
//   message: alpha * xh[j]; aggr 'add'; concat heads (or mean for concat=False) + bias
//
// Mapping: one wave64 per destination row (forward, K6a) or per source column (K6b).
// Edge/head pairs of a row are spread over lanes with the head fixed per lane
// (lane & (H-1), H a power of two <= 64), so per-head max / sum / dot reductions are
// xor-shuffles over lane offsets >= H — no LDS, no atomics.  Attention weights are
// recomputed (bit-identically) in the feature pass instead of being re-read.
#include <algorithm>
#include <initializer_list>
#include <utility>

#include "gemm_common.hpp"  // keep_elem (the counter-hash dropout shared with the NT epilogue)

namespace gnnmp {
namespace {

__device__ __forceinline__ float leaky(float z, float slope) { return z > 0.0f ? z : z * slope; }

// Fast-path arithmetic (lane-group kernels): exp as one v_exp_f32 of x*log2(e) (exp(-inf) = 0,
// relative error ~|x| * 2^-24: the softmax arguments are <= 0 and large |x| carry negligible
// weight), 1/x as one v_rcp_f32 (1 ulp).  Both well inside the 1e-5 parity bound.
__device__ __forceinline__ float fexp(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }
__device__ __forceinline__ float frcp(float x) { return __builtin_amdgcn_rcpf(x); }
// 24-bit row offsets (the host routes graphs with N or a row pitch >= 2^24 to the generic kernels)
__device__ __forceinline__ uint32_t roff(int32_t row, int64_t ld) { return __umul24((uint32_t)row, (uint32_t)ld); }

__device__ __forceinline__ float wave_max_over_heads(float v, int H) {
  for (int off = 32; off >= H; off >>= 1) v = fmaxf(v, __shfl_xor(v, off));
  return v;
}
__device__ __forceinline__ float wave_sum_over_heads(float v, int H) {
  for (int off = 32; off >= H; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

__global__ __launch_bounds__(256) void gat_scores_kernel(int64_t N, int32_t H, int32_t C,
                                                         const float* __restrict__ xh, int64_t ld,
                                                         const float* __restrict__ att_s,
                                                         const float* __restrict__ att_d,
                                                         float* __restrict__ a_s, float* __restrict__ a_d) {
  int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= N * H) return;
  int64_t n = t / H;
  int h = (int)(t % H);
  const float* xr = xh + n * ld + (int64_t)h * C;
  const float* as = att_s + (int64_t)h * C;
  const float* ad = att_d + (int64_t)h * C;
  float s = 0.0f, d = 0.0f;
  for (int c = 0; c < C; ++c) {
    float v = xr[c];
    s += v * as[c];
    d += v * ad[c];
  }
  a_s[t] = s;
  a_d[t] = d;
}

struct GatArgs {
  const int32_t* rowptr; const int32_t* col;
  const int32_t* colptr; const int32_t* row; const int32_t* csc2csr;
  int64_t N;
  int32_t H, C, concat;
  float slope;
  const float* xh; int64_t ld_xh;
  const float* a_s; const float* a_d;
  const float* bias;
  float* alpha;
  float* out; int64_t ldo;
  // backward
  const float* att_s; const float* att_d;
  const float* dout; int64_t ld_dout;
  float* dz;      // [S, H]
  float* dad;     // [N, H]
  float* das;     // [N, H]
  float* dxh; int64_t ld_dxh;
  // explain mode (generic kernels only): per-CSR-slot message multiplier and its gradient
  const float* ew;  // [S] or null
  float* dew;       // [S] or null
  // the CSR group passes in the plan's degree order (K0b csr_split order: position -> row; rows
  // of one wave then have nearly the same slot count and walk in lockstep), null: row order
  const int32_t* order;
  // rows pass with the hidden layer's store backward fused (gnn_gat_bwd_act_f32): dout holds dy,
  // d pre = dy * keep / (1-p) * elu'(pre) is formed from it and the stored y = dropout(elu(pre))
  // as each row's slice is loaded, and written to dpre for the cols pass
  const float* y; int64_t ld_y;
  float* dpre; int64_t ld_dpre;
  int32_t pe_act, pe_drop; uint32_t pe_thresh; float pe_scale, pe_keep;
  uint64_t pe_seed; const uint64_t* pe_seed_ptr;
  // (ABI 24) dy given as dz · proj (dz [N, pnproj], proj [pnproj, F]): the output conv's lin
  // backward formed as each row slice loads — GATNet's dh is never materialised
  const float* pdz; int64_t ld_pdz; const float* pproj; int32_t pnproj;
  // (ABI 25) float bits of max |dxh| per GNN_ROWMAX_ROWS-row group: zeroed by the rows pass,
  // atomicMax'd by the cols pass as it stores dxh (max is order-free: deterministic)
  uint32_t* dxh_rowmax;
};

// the row of group position pos (pos < N)
__device__ __forceinline__ int64_t gat_row(const GatArgs& a, int64_t pos) {
  return (a.order && pos < a.N) ? (int64_t)a.order[pos] : pos;
}

// ---------------------------------------------------------------- forward (K5)
__global__ __launch_bounds__(256) void gat_fwd_kernel(GatArgs a) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int H = a.H, C = a.C;
  const int hl = lane & (H - 1);  // this lane's head in the pair loops
  for (int64_t r = (int64_t)blockIdx.x * 4 + wave; r < a.N; r += (int64_t)gridDim.x * 4) {
    const int32_t beg = __builtin_amdgcn_readfirstlane(a.rowptr[r]);
    const int32_t end = __builtin_amdgcn_readfirstlane(a.rowptr[r + 1]);
    const int32_t npair = (end - beg) * H;
    const float adr = a.a_d[r * H + hl];
    // pass 1: per-head max of e
    float m = -INFINITY;
    for (int32_t idx = lane; idx < npair; idx += 64) {
      int32_t k = beg + idx / H;
      float e = leaky(a.a_s[(int64_t)a.col[k] * H + hl] + adr, a.slope);
      m = fmaxf(m, e);
    }
    m = wave_max_over_heads(m, H);
    // pass 2: per-head sum of exp
    float s = 0.0f;
    for (int32_t idx = lane; idx < npair; idx += 64) {
      int32_t k = beg + idx / H;
      float e = leaky(a.a_s[(int64_t)a.col[k] * H + hl] + adr, a.slope);
      s += expf(e - m);
    }
    s = wave_sum_over_heads(s, H);
    const float denom = s + 1e-16f;
    // pass 3: alpha per slot (saved for backward)
    for (int32_t idx = lane; idx < npair; idx += 64) {
      int32_t k = beg + idx / H;
      float e = leaky(a.a_s[(int64_t)a.col[k] * H + hl] + adr, a.slope);
      a.alpha[(int64_t)k * H + hl] = expf(e - m) / denom;
    }
    // pass 4: features.  lane f gathers alpha_k,h(f) * xh[j_k, f]
    if (a.concat) {
      const int F = H * C;
      for (int f = lane; f < F; f += 64) {
        const int h = f / C;
        const float mh = __shfl(m, h);
        const float dh = __shfl(denom, h);
        const float adh = a.a_d[r * H + h];
        float acc = 0.0f;
        for (int32_t k = beg; k < end; ++k) {
          int32_t j = a.col[k];
          float e = leaky(a.a_s[(int64_t)j * H + h] + adh, a.slope);
          float al = expf(e - mh) / dh;
          if (a.ew) al *= a.ew[k];
          acc += al * a.xh[(int64_t)j * a.ld_xh + f];
        }
        if (a.bias) acc += a.bias[f];
        a.out[r * a.ldo + f] = acc;
      }
    } else {
      for (int c = lane; c < C; c += 64) {
        float tot = 0.0f;
        for (int h = 0; h < H; ++h) {
          const float mh = __shfl(m, h);
          const float dh = __shfl(denom, h);
          const float adh = a.a_d[r * H + h];
          float acc = 0.0f;
          for (int32_t k = beg; k < end; ++k) {
            int32_t j = a.col[k];
            float e = leaky(a.a_s[(int64_t)j * H + h] + adh, a.slope);
            float al = expf(e - mh) / dh;
            if (a.ew) al *= a.ew[k];
            acc += al * a.xh[(int64_t)j * a.ld_xh + h * C + c];
          }
          tot += acc;
        }
        tot = tot / (float)H;
        if (a.bias) tot += a.bias[c];
        a.out[r * a.ldo + c] = tot;
      }
    }
  }
}

// d out[r, h, c] as the per-head upstream gradient (mean over heads divides by H).
__device__ __forceinline__ float dO(const GatArgs& a, int64_t r, int h, int c) {
  if (a.concat) return a.dout[r * a.ld_dout + (int64_t)h * a.C + c];
  return a.dout[r * a.ld_dout + c] / (float)a.H;
}

// ---------------------------------------------------------------- backward K6a (CSR rows)
__global__ __launch_bounds__(256) void gat_bwd_rows_kernel(GatArgs a) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int H = a.H, C = a.C;
  const int hl = lane & (H - 1);
  for (int64_t r = (int64_t)blockIdx.x * 4 + wave; r < a.N; r += (int64_t)gridDim.x * 4) {
    const int32_t beg = __builtin_amdgcn_readfirstlane(a.rowptr[r]);
    const int32_t end = __builtin_amdgcn_readfirstlane(a.rowptr[r + 1]);
    const int32_t npair = (end - beg) * H;
    const float adr = a.a_d[r * H + hl];
    // t_h = sum_k alpha_k * dalpha_k
    float t = 0.0f;
    for (int32_t idx = lane; idx < npair; idx += 64) {
      int32_t k = beg + idx / H;
      int32_t j = a.col[k];
      const float* xr = a.xh + (int64_t)j * a.ld_xh + (int64_t)hl * C;
      float da = 0.0f;
      for (int c = 0; c < C; ++c) da += dO(a, r, hl, c) * xr[c];
      if (a.ew) da *= a.ew[k];
      t += a.alpha[(int64_t)k * H + hl] * da;
    }
    t = wave_sum_over_heads(t, H);
    float sdz = 0.0f;
    for (int32_t idx = lane; idx < npair; idx += 64) {
      int32_t k = beg + idx / H;
      int32_t j = a.col[k];
      const float* xr = a.xh + (int64_t)j * a.ld_xh + (int64_t)hl * C;
      float da = 0.0f;
      for (int c = 0; c < C; ++c) da += dO(a, r, hl, c) * xr[c];
      float al = a.alpha[(int64_t)k * H + hl];
      if (a.dew) {  // d ew[k] = sum over heads of alpha * <dO, xh[j]>: the H lanes of slot k are adjacent
        float v = al * da;
        for (int off = 1; off < H; off <<= 1) v += __shfl_xor(v, off);
        if (hl == 0) a.dew[k] = v;
      }
      if (a.ew) da *= a.ew[k];
      float de = al * (da - t);
      float z = a.a_s[(int64_t)j * H + hl] + adr;
      float dzv = z > 0.0f ? de : de * a.slope;
      a.dz[(int64_t)k * H + hl] = dzv;
      sdz += dzv;
    }
    sdz = wave_sum_over_heads(sdz, H);
    if (lane < H) a.dad[r * H + lane] = sdz;
  }
}

// ---------------------------------------------------------------- backward K6b (CSC columns)
__global__ __launch_bounds__(256) void gat_bwd_cols_kernel(GatArgs a) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int H = a.H, C = a.C;
  const int hl = lane & (H - 1);
  const int F = H * C;
  for (int64_t j = (int64_t)blockIdx.x * 4 + wave; j < a.N; j += (int64_t)gridDim.x * 4) {
    const int32_t beg = __builtin_amdgcn_readfirstlane(a.colptr[j]);
    const int32_t end = __builtin_amdgcn_readfirstlane(a.colptr[j + 1]);
    const int32_t npair = (end - beg) * H;
    float s = 0.0f;
    for (int32_t idx = lane; idx < npair; idx += 64) {
      int32_t k = beg + idx / H;
      s += a.dz[(int64_t)a.csc2csr[k] * H + hl];
    }
    s = wave_sum_over_heads(s, H);  // d a_src[j, hl]
    if (lane < H) a.das[j * H + lane] = s;
    for (int f = lane; f < F; f += 64) {
      const int h = f / C;
      const int c = f - h * C;
      float acc = 0.0f;
      for (int32_t k = beg; k < end; ++k) {
        int32_t i = a.row[k];
        const int32_t ks = a.csc2csr[k];
        float al = a.alpha[(int64_t)ks * H + h];
        if (a.ew) al *= a.ew[ks];
        acc += al * dO(a, i, h, c);
      }
      const float dash = __shfl(s, h);
      const float dadh = a.dad[j * H + h];
      acc += dash * a.att_s[f] + dadh * a.att_d[f];
      a.dxh[j * a.ld_dxh + f] = acc;
    }
  }
}

// d att[f] = sum_n dscore[n, h(f)] * xh[n, f]  (two-stage, deterministic)
constexpr int kAttBlocks = 512;  // generic path partials
__global__ __launch_bounds__(256) void gat_att_partial_kernel(GatArgs a, int64_t rows_per_blk, float* part) {
  const int F = a.H * a.C;
  int64_t r0 = blockIdx.x * rows_per_blk;
  int64_t r1 = r0 + rows_per_blk < a.N ? r0 + rows_per_blk : a.N;
  for (int f = threadIdx.x; f < F; f += blockDim.x) {
    const int h = f / a.C;
    float ss = 0.0f, sd = 0.0f;
    for (int64_t n = r0; n < r1; ++n) {
      float x = a.xh[n * a.ld_xh + f];
      ss += a.das[n * a.H + h] * x;
      sd += a.dad[n * a.H + h] * x;
    }
    part[((int64_t)blockIdx.x * 2 + 0) * F + f] = ss;
    part[((int64_t)blockIdx.x * 2 + 1) * F + f] = sd;
  }
}

__global__ void gat_att_final_kernel(int F, int nblk, const float* part, float* d_att_s, float* d_att_d) {
  int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= F) return;
  float ss = 0.0f, sd = 0.0f;
  for (int b = 0; b < nblk; ++b) {
    ss += part[((int64_t)b * 2 + 0) * F + f];
    sd += part[((int64_t)b * 2 + 1) * F + f];
  }
  d_att_s[f] = ss;
  d_att_d[f] = sd;
}


// ================================================================ lane-group kernels (fast path)
// A destination row (forward, rows pass) or source column (cols pass) is owned by a group of
// G lanes (G a power of two, 4..64), so a wave64 serves 64/G rows at once instead of idling
// most lanes on Elliptic's ~2-slot rows.  Two lane views of the same group:
//   pair view:  lane lig walks (slot, head) pairs idx = lig + t*G with head lig & (H-1) fixed
//               (G % H == 0), so per-head max / sum are xor-shuffles over offsets H..G/2;
//   slot view:  lane lig owns VEC consecutive features fl*VEC.. (fl = lig & (FLp-1), all of one
//               head) and walks the slots k = beg + ep, step EP = G/FLp; partial sums over the
//               EP edge phases are xor-shuffles over offsets FLp..G/2.
// The softmax statistics of head h live in lane h of the group after the pair-view
// reduction and reach the slot view through one __shfl (the whole wave participates).
struct GatGeom {
  int G, lgG;    // lanes per row/column (slot view and forward pair view)
  int Gb, lgGb;  // lanes per row in the backward rows pass (pair view only)
  int lgH;
  int FL, FLp, lgFLp;  // feature slots of VEC floats, its power-of-two ceiling
  int L;               // slots per head (C / VEC)
};

template <int VEC>
struct VecF { float v[VEC]; };

template <int VEC>
__device__ __forceinline__ VecF<VEC> ldv(const float* p) {
  VecF<VEC> r;
  if constexpr (VEC == 4) {
    float4 t = *reinterpret_cast<const float4*>(p);
    r.v[0] = t.x; r.v[1] = t.y; r.v[2] = t.z; r.v[3] = t.w;
  } else if constexpr (VEC == 2) {
    float2 t = *reinterpret_cast<const float2*>(p);
    r.v[0] = t.x; r.v[1] = t.y;
  } else {
    r.v[0] = *p;
  }
  return r;
}

template <int VEC>
__device__ __forceinline__ void stv(float* p, const VecF<VEC>& r) {
  if constexpr (VEC == 4) *reinterpret_cast<float4*>(p) = make_float4(r.v[0], r.v[1], r.v[2], r.v[3]);
  else if constexpr (VEC == 2) *reinterpret_cast<float2*>(p) = make_float2(r.v[0], r.v[1]);
  else *p = r.v[0];
}

// Long rows: the plan's K0b csr_split lists the rows with more than T slots (Elliptic's hubs).
// A group of G lanes would walk such a row in one dependent loop and set the kernel's tail,
// so each long row gets a whole 256-thread block, and those blocks are dispatched ahead of
// the short-row blocks (blockIdx < n): their chains overlap the bulk instead of trailing it.
// The short-row path skips rows with more than T slots.
struct GatLong {
  const int32_t* rows;
  int32_t n;
  int32_t T;
};

// Store-side operands of the forward: GATNet's hidden-layer activation and dropout
// (gnn.py:73-74) and, for the in-kernel score form, the attention vectors and score outputs.
struct GatEpi {
  int act;              // gnn_act
  int dropout;
  uint32_t keep_thresh;
  float drop_scale;
  uint64_t seed;        // as NTArgs: *seed_ptr * golden + seed when seed_ptr is set
  const uint64_t* seed_ptr;
  float* as_out;        // XS: a_src / a_dst written [N, H]
  float* ad_out;
  // (ABI 24, concat layers) z = out · projᵀ beside the store: GATNet's output conv's lin on the
  // hidden layer's stored rows (proj [nproj, F], nproj <= 4)
  const float* proj; int32_t nproj; float* z; int64_t ldz;
};


__device__ __forceinline__ uint64_t gat_seed(const GatEpi& e) {
  return e.seed_ptr ? (*e.seed_ptr) * 0x9E3779B97F4A7C15ull + e.seed : e.seed;
}

__device__ __forceinline__ float gat_store_val(const GatEpi& e, uint64_t seed, float v, int64_t r, int col, int Fo) {
  if (e.act == GNN_ACT_ELU) v = v > 0.0f ? v : expm1f(v);  // F.elu: expm1 (no cancellation near 0)
  if (e.dropout)
    v = keep_elem(seed, (uint32_t)r * (uint32_t)Fo + (uint32_t)col, e.keep_thresh) ? v * e.drop_scale : 0.0f;
  return v;
}

// Sum of a per-lane partial over the L slot-view lanes of one head (contiguous, starting at
// lane h0 of the wave).  L a power of two: xor butterfly (commutative pairs: every lane gets the
// bit-identical sum); otherwise a fixed-order gather.  All lanes of the head must be active.
__device__ __forceinline__ float head_sum(float v, int L, int h0) {
  if ((L & (L - 1)) == 0) {
    for (int off = 1; off < L; off <<= 1) v += __shfl_xor(v, off);
    return v;
  }
  float s = 0.0f;
  for (int i = 0; i < L; ++i) s += __shfl(v, h0 + i);
  return s;
}

template <int VEC>
__device__ __forceinline__ float vdot(const VecF<VEC>& x, const VecF<VEC>& w) {
  float s = x.v[0] * w.v[0];
#pragma unroll
  for (int i = 1; i < VEC; ++i) s = fmaf(x.v[i], w.v[i], s);
  return s;
}

// z[r, q] = Σ_f o[f] · proj[q, f] over the row's stored slice: each phase-0 lane its VEC features
// (pw: the lane's slice of proj's rows), summed over the FLp lanes of the row — the phase-0 lanes
// of a group are its lanes 0 .. FLp - 1.  FLp == 16 (GATNet's 64-wide hidden rows at VEC 4): the
// row is one DPP row, summed by two quad_perm steps and row_shr 4 / 8 into its lane 15 (no LDS
// crossbar round trips); otherwise an xor butterfly, lane 0 holding the sum.  Every lane of the wave
// calls it (lanes without a stored slice contribute 0); `own`: the row is this group's to store.
template <int VEC, int NP>
__device__ __forceinline__ void gat_store_proj(const GatEpi& e, const VecF<VEC>& o, bool on, const VecF<VEC> (&pw)[NP],
                                               int FLp, int64_t r, bool own, int fl) {
  float pz[NP];
#pragma unroll
  for (int q = 0; q < NP; ++q) pz[q] = on ? vdot<VEC>(o, pw[q]) : 0.f;
  int wl = 0;
  if (FLp == 16) {
    wl = 15;
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      float v = pz[q];
      v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, true));   // quad_perm 1,0,3,2
      v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, true));   // quad_perm 2,3,0,1
      v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x114, 0xF, 0xF, true));  // row_shr:4
      v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x118, 0xF, 0xF, true));  // row_shr:8
      pz[q] = v;
    }
  } else {
    for (int off = 1; off < FLp; off <<= 1) {
#pragma unroll
      for (int q = 0; q < NP; ++q) pz[q] += __shfl_xor(pz[q], off);
    }
  }
  if (own && fl == wl) {
#pragma unroll
    for (int q = 0; q < NP; ++q)
      if (q < e.nproj) e.z[r * e.ldz + q] = pz[q];
  }
}
// the lane's slice of proj's first NP rows (zeros past nproj or for lanes without a feature slot)
template <int VEC, int NP>
__device__ __forceinline__ void gat_load_proj(const GatEpi& e, bool ok, int F, int f0, VecF<VEC> (&pw)[NP]) {
#pragma unroll
  for (int q = 0; q < NP; ++q) {
#pragma unroll
    for (int i = 0; i < VEC; ++i) pw[q].v[i] = 0.f;
    if (ok && q < e.nproj) pw[q] = ldv<VEC>(e.proj + (int64_t)q * F + f0);
  }
}

// Online softmax state of one slot-view lane: running max m, sum s and accumulator (both
// scaled by exp(-m)).  merge() combines two states; it is symmetric, so the two lanes of an
// xor exchange end with bit-identical results.
template <int VEC>
struct Online {
  float m, s;
  VecF<VEC> acc;
  __device__ __forceinline__ void init() {
    m = -INFINITY;
    s = 0.0f;
#pragma unroll
    for (int i = 0; i < VEC; ++i) acc.v[i] = 0.0f;
  }
  // two slots at once (e1 = -inf: absent): 3 exps per pair; returns their unnormalised weights
  __device__ __forceinline__ void add2(float e0, const VecF<VEC>& x0, float e1, const VecF<VEC>& x1, float& p0,
                                       float& p1) {
    const float mn = fmaxf(m, fmaxf(e0, e1));
    const float sc = fexp(m - mn);  // 0 while m = -inf
    p0 = fexp(e0 - mn);
    p1 = fexp(e1 - mn);
    s = (s * sc + p0) + p1;
#pragma unroll
    for (int i = 0; i < VEC; ++i) acc.v[i] = (acc.v[i] * sc + p0 * x0.v[i]) + p1 * x1.v[i];
    m = mn;
  }
  __device__ __forceinline__ void merge(float m2, float s2, const VecF<VEC>& acc2) {
    const float mn = fmaxf(m, m2);
    const float c1 = m == -INFINITY ? 0.0f : fexp(m - mn);
    const float c2 = m2 == -INFINITY ? 0.0f : fexp(m2 - mn);
    s = s * c1 + s2 * c2;
#pragma unroll
    for (int i = 0; i < VEC; ++i) acc.v[i] = acc.v[i] * c1 + acc2.v[i] * c2;
    m = mn;
  }
};

// Per-lane geometry of the slot view (lanes over VEC-float feature slots x slot phases).
struct SlotLane {
  int fl, ep, EP, f0, hs, c0, L, hfirst;  // hfirst: first lane (wave index) of this lane's head
  bool ok;
};

__device__ __forceinline__ SlotLane slot_lane(const GatGeom& g, int lig, int width, int wave_lane, int VEC, int C) {
  SlotLane s;
  s.fl = lig & (g.FLp - 1);
  s.ep = lig >> g.lgFLp;
  s.EP = width >> g.lgFLp;
  s.ok = s.fl < g.FL;
  s.f0 = s.fl * VEC;
  s.hs = s.ok ? s.f0 / C : 0;
  s.c0 = s.f0 - s.hs * C;
  s.L = g.L;
  s.hfirst = (wave_lane - s.fl) + s.hs * s.L;
  return s;
}

// The slot pass of one lane: slots beg + ep, += EP, two per trip (both neighbour rows in flight;
// the lanes of a head share their trip count, so the head_sum exchanges stay converged).  The
// first trip's weights stay in registers (p0f, p1f with the running max m1 they refer to: most
// rows end there); later trips park their raw scores in alpha (writer lane) for normalise_alpha.
template <int VEC, bool XS>
__device__ __forceinline__ void slot_pass(const GatArgs& a, const SlotLane& sl, int32_t beg, int32_t end, float adr,
                                          const VecF<VEC>& as_v, bool writer, Online<VEC>& st, float& p0f,
                                          float& p1f, float& m1) {
  const int H = a.H;
  const int32_t k0 = beg + sl.ep;
  for (int32_t k = k0; k < end; k += 2 * sl.EP) {
    const bool two = k + sl.EP < end;
    const int32_t j0 = a.col[k];
    const int32_t j1 = a.col[two ? k + sl.EP : k];  // unconditional (clamped) load: no join wait
    const VecF<VEC> x0 = ldv<VEC>(a.xh + roff(j0, a.ld_xh) + sl.f0);
    const VecF<VEC> x1 = ldv<VEC>(a.xh + roff(j1, a.ld_xh) + sl.f0);
    float s0, s1;
    if constexpr (XS) {
      s0 = head_sum(vdot<VEC>(x0, as_v), sl.L, sl.hfirst);
      s1 = head_sum(vdot<VEC>(x1, as_v), sl.L, sl.hfirst);
    } else {
      s0 = a.a_s[roff(j0, H) + sl.hs];
      s1 = a.a_s[roff(j1, H) + sl.hs];
    }
    const float e0 = leaky(s0 + adr, a.slope);
    const float e1 = two ? leaky(s1 + adr, a.slope) : -INFINITY;
    float p0, p1;
    st.add2(e0, x0, e1, x1, p0, p1);
    if (k == k0) {
      p0f = p0;
      p1f = p1;
      m1 = st.m;
    } else if (writer) {
      a.alpha[roff(k, H) + sl.hs] = e0;
      if (two) a.alpha[roff(k + sl.EP, H) + sl.hs] = e1;
    }
  }
}

// alpha = exp(e - m) / denom for the writer lane's slots (rinv = 1 / denom): the first trip as
// its kept weights rescaled to the final max, later trips from their parked raw scores.
__device__ __forceinline__ void normalise_alpha(const GatArgs& a, const SlotLane& sl, int32_t beg, int32_t end,
                                                float p0f, float p1f, float m1, float m, float rinv) {
  const int H = a.H;
  const int32_t k0 = beg + sl.ep;
  if (k0 < end) {
    const float sc = fexp(m1 - m) * rinv;
    a.alpha[roff(k0, H) + sl.hs] = p0f * sc;
    if (k0 + sl.EP < end) a.alpha[roff(k0 + sl.EP, H) + sl.hs] = p1f * sc;
  }
#pragma unroll 1
  for (int32_t k = k0 + 2 * sl.EP; k < end; k += sl.EP) {
    float* p = a.alpha + roff(k, H) + sl.hs;
    *p = fexp(*p - m) * rinv;
  }
}

constexpr int kLongLds = 4 * 64 * 2 + 4 * 256 + 256;  // wave m/s [4][64] x 2, partials [4][256], final [256]

// One block, one long row (more than T slots): 256/FLp slot phases, each lane an online
// softmax over its slots; phases merged in the wave by xor exchanges, waves through LDS in a
// fixed order.  XS: scores from the gathered xh rows (and the row's own a_src / a_dst written).
template <int VEC, bool XS>
__device__ void gat_fwd_long_row(const GatArgs& a, const GatGeom& g, const GatEpi& ep_, uint64_t seed,
                                 const VecF<VEC>& as_v, const VecF<VEC>& ad_v, int64_t r, float* sh) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int H = a.H, C = a.C, F = H * C;
  const int Fo = a.concat ? F : C;
  const SlotLane sl = slot_lane(g, tid, 256, lane, VEC, C);
  const int32_t beg = a.rowptr[r], end = a.rowptr[r + 1];
  float* sm = sh;
  float* ss = sh + 256;
  float* red = sh + 512;
  float* fin = sh + 512 + 1024;
  float adr;
  if constexpr (XS) {
    VecF<VEC> xr;
#pragma unroll
    for (int i = 0; i < VEC; ++i) xr.v[i] = 0.0f;
    if (sl.ok) xr = ldv<VEC>(a.xh + roff((int32_t)r, a.ld_xh) + sl.f0);
    const float ps = head_sum(vdot<VEC>(xr, as_v), sl.L, sl.hfirst);
    adr = head_sum(vdot<VEC>(xr, ad_v), sl.L, sl.hfirst);
    if (sl.ok && sl.ep == 0 && sl.fl == sl.hs * sl.L) {
      ep_.as_out[r * H + sl.hs] = ps;
      ep_.ad_out[r * H + sl.hs] = adr;
    }
  } else {
    adr = a.a_d[r * H + sl.hs];
  }
  const bool writer = sl.ok && sl.fl == sl.hs * sl.L;  // one lane per (head, phase) keeps the raw scores
  Online<VEC> st;
  st.init();
  float p0f = 0.0f, p1f = 0.0f, m1 = 0.0f;
  if (sl.ok) slot_pass<VEC, XS>(a, sl, beg, end, adr, as_v, writer, st, p0f, p1f, m1);
  for (int off = 32; off >= g.FLp; off >>= 1) {
    VecF<VEC> a2;
#pragma unroll
    for (int i = 0; i < VEC; ++i) a2.v[i] = __shfl_xor(st.acc.v[i], off);
    st.merge(__shfl_xor(st.m, off), __shfl_xor(st.s, off), a2);
  }
  if (lane < g.FLp) {
    sm[wave * 64 + sl.fl] = st.m;
    ss[wave * 64 + sl.fl] = st.s;
    if (sl.ok) {
#pragma unroll
      for (int i = 0; i < VEC; ++i) red[wave * 256 + sl.f0 + i] = st.acc.v[i];
    }
  }
  __syncthreads();
  Online<VEC> tot;
  tot.init();
  if (sl.ok) {
    for (int w = 0; w < 4; ++w) {
      VecF<VEC> a2;
#pragma unroll
      for (int i = 0; i < VEC; ++i) a2.v[i] = red[w * 256 + sl.f0 + i];
      tot.merge(sm[w * 64 + sl.fl], ss[w * 64 + sl.fl], a2);
    }
  }
  const float rinv = frcp(tot.s + 1e-16f);
  if (a.concat) {
    VecF<VEC> o;
#pragma unroll
    for (int i = 0; i < VEC; ++i) o.v[i] = 0.0f;
    if (sl.ok && sl.ep == 0) {
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        const int f = sl.f0 + i;
        o.v[i] = gat_store_val(ep_, seed, tot.acc.v[i] * rinv + (a.bias ? a.bias[f] : 0.0f), r, f, Fo);
      }
      stv<VEC>(a.out + r * a.ldo + sl.f0, o);
    }
    // (the row's phase-0 lanes are threads 0 .. FLp - 1 of wave 0)
    if (ep_.nproj > 0) {
      VecF<VEC> pw[2];
      gat_load_proj<VEC, 2>(ep_, sl.ok && sl.ep == 0, F, sl.f0, pw);
      gat_store_proj<VEC, 2>(ep_, o, sl.ok && sl.ep == 0, pw, g.FLp, r, wave == 0 && sl.ep == 0, sl.fl);
    }
  } else {
    if (sl.ok && sl.ep == 0) {
#pragma unroll
      for (int i = 0; i < VEC; ++i) fin[sl.f0 + i] = tot.acc.v[i] * rinv;
    }
    __syncthreads();
    for (int c = tid; c < C; c += 256) {
      float t = 0.0f;
      for (int h = 0; h < H; ++h) t += fin[h * C + c];
      a.out[r * a.ldo + c] = gat_store_val(ep_, seed, t / (float)H + (a.bias ? a.bias[c] : 0.0f), r, c, Fo);
    }
  }
  if (writer) normalise_alpha(a, sl, beg, end, p0f, p1f, m1, tot.m, rinv);
}

// Forward, short rows (<= T slots): G lanes per row in the slot view, one pass with an online
// softmax per lane, merged across the EP slot phases by xor exchanges; out = acc / (s + 1e-16)
// (+ bias, activation, dropout).  The lane that owns a (head, phase) normalises each slot's raw
// score into alpha afterwards (the first trip's from registers, later ones re-read from alpha).
// XS: the scores come from the gathered xh rows themselves (a_src[j] = <xh[j,h,:], att_src[h]>,
// reduced over the head's lanes), so the only dependent loads per row are rowptr -> col -> xh.
template <int VEC, bool XS>
__global__ __launch_bounds__(256) void gat_fwd_group_kernel(GatArgs a, GatGeom g, GatLong lg, GatEpi ep_) {
  __shared__ float sh[kLongLds];
  __shared__ float psh[2 * 256];  // the store's projection rows (ep_.nproj > 0: proj [nproj <= 2][F <= 256])
  const int lane = threadIdx.x & 63;
  const int H = a.H, C = a.C, F = H * C;
  if (ep_.nproj > 0) {  // (block-uniform, before the long-row split)
    for (int i = threadIdx.x; i < 2 * F; i += 256) psh[(i / F) * 256 + i % F] = i / F < ep_.nproj ? ep_.proj[i] : 0.f;
    __syncthreads();
  }
  const int Fo = a.concat ? F : C;
  const uint64_t seed = ep_.dropout ? gat_seed(ep_) : 0;
  // attention vectors of this lane's feature slot (XS)
  VecF<VEC> as_v, ad_v;
#pragma unroll
  for (int i = 0; i < VEC; ++i) { as_v.v[i] = 0.0f; ad_v.v[i] = 0.0f; }
  if ((int)blockIdx.x < lg.n) {
    const SlotLane sl = slot_lane(g, threadIdx.x, 256, lane, VEC, C);
    if (XS && sl.ok) { as_v = ldv<VEC>(a.att_s + sl.f0); ad_v = ldv<VEC>(a.att_d + sl.f0); }
    gat_fwd_long_row<VEC, XS>(a, g, ep_, seed, as_v, ad_v, lg.rows[blockIdx.x], sh);
    return;
  }
  const int64_t bid = blockIdx.x - lg.n, nblk = gridDim.x - lg.n;
  const int wave = threadIdx.x >> 6;
  const int G = g.G;
  const int lig = lane & (G - 1);
  const int rpw = 64 >> g.lgG;
  const SlotLane sl = slot_lane(g, lig, G, lane, VEC, C);
  if (XS && sl.ok) { as_v = ldv<VEC>(a.att_s + sl.f0); ad_v = ldv<VEC>(a.att_d + sl.f0); }
  const bool writer = sl.ok && sl.fl == sl.hs * sl.L;
  const int64_t rpb = 4 * (int64_t)rpw;
  for (int64_t base = bid * rpb; base < a.N; base += nblk * rpb) {
    const int64_t r = gat_row(a, base + wave * rpw + (lane >> g.lgG));
    int32_t beg = 0, end = 0;
    if (r < a.N) { beg = a.rowptr[r]; end = a.rowptr[r + 1]; }
    const bool own = r < a.N && end - beg <= lg.T;
    if (!own) end = beg;
    float adr;
    if constexpr (XS) {
      VecF<VEC> xr;
#pragma unroll
      for (int i = 0; i < VEC; ++i) xr.v[i] = 0.0f;
      if (r < a.N && sl.ok) xr = ldv<VEC>(a.xh + roff((int32_t)r, a.ld_xh) + sl.f0);  // beside the rowptr loads
      const float ps = head_sum(vdot<VEC>(xr, as_v), sl.L, sl.hfirst);
      adr = head_sum(vdot<VEC>(xr, ad_v), sl.L, sl.hfirst);
      if (own && sl.ep == 0 && writer) {
        ep_.as_out[r * H + sl.hs] = ps;
        ep_.ad_out[r * H + sl.hs] = adr;
      }
    } else {
      adr = a.a_d[(own ? r : 0) * H + sl.hs];
      adr = own ? adr : 0.0f;
    }
    Online<VEC> st;
    st.init();
    float p0f = 0.0f, p1f = 0.0f, m1 = 0.0f;
    if (sl.ok) slot_pass<VEC, XS>(a, sl, beg, end, adr, as_v, writer, st, p0f, p1f, m1);
    for (int off = G >> 1; off >= g.FLp; off >>= 1) {
      VecF<VEC> a2;
#pragma unroll
      for (int i = 0; i < VEC; ++i) a2.v[i] = __shfl_xor(st.acc.v[i], off);
      st.merge(__shfl_xor(st.m, off), __shfl_xor(st.s, off), a2);
    }
    const float rinv = frcp(st.s + 1e-16f);
    VecF<VEC> o;
#pragma unroll
    for (int i = 0; i < VEC; ++i) o.v[i] = st.acc.v[i] * rinv;
    if (!a.concat) {  // mean over heads: same channel sits L slots apart (L, H powers of two)
      for (int off = g.FLp >> 1; off >= g.L; off >>= 1) {
#pragma unroll
        for (int i = 0; i < VEC; ++i) o.v[i] += __shfl_xor(o.v[i], off);
      }
    }
    const bool stor = own && sl.ok && sl.ep == 0;
    if (a.concat && ep_.nproj > 0) {  // (wave-uniform) the stored rows' projection z = out · projᵀ
      if (stor) {
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
          const int f = sl.f0 + i;
          o.v[i] = gat_store_val(ep_, seed, o.v[i] + (a.bias ? a.bias[f] : 0.0f), r, f, Fo);
        }
        stv<VEC>(a.out + r * a.ldo + sl.f0, o);
      }
      VecF<VEC> pw[2];  // the lane's slice of the projection rows, from LDS (no registers held across rows)
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int i = 0; i < VEC; ++i) pw[q].v[i] = sl.ok ? psh[q * 256 + sl.f0 + i] : 0.f;
      gat_store_proj<VEC, 2>(ep_, o, stor, pw, g.FLp, r, stor, sl.fl);
    } else if (stor) {
      if (a.concat) {
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
          const int f = sl.f0 + i;
          o.v[i] = gat_store_val(ep_, seed, o.v[i] + (a.bias ? a.bias[f] : 0.0f), r, f, Fo);
        }
        stv<VEC>(a.out + r * a.ldo + sl.f0, o);
      } else if (sl.hs == 0) {
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
          const int c = sl.c0 + i;
          o.v[i] = gat_store_val(ep_, seed, o.v[i] / (float)H + (a.bias ? a.bias[c] : 0.0f), r, c, Fo);
        }
        stv<VEC>(a.out + r * a.ldo + sl.c0, o);
      }
    }
    if (writer) normalise_alpha(a, sl, beg, end, p0f, p1f, m1, st.m, rinv);
  }
}

// Backward rows pass in the slot view (the forward's lanes): for slot k of row r and head h,
// d alpha = <dO[r,h,:], xh[j,h,:]> (a VEC-wide dot per lane, summed over the head's lanes),
// t_h = sum_k alpha d alpha (merged over the EP phases), then d e = alpha (d alpha - t), the
// leaky-relu backward into dz[k,h] and d a_dst[r,h] = sum_k dz.  The first trip's
// (d alpha, alpha, score sign) stay in registers; later trips park d alpha in dz (writer lane).
struct BwdSlot {
  float da, al;
  bool pos;
};

template <int VEC>
__device__ __forceinline__ float bwd_pass1(const GatArgs& a, const SlotLane& sl, int32_t beg, int32_t end, float adr,
                                           const VecF<VEC>& dO, float inv_h, bool writer, BwdSlot& q0, BwdSlot& q1) {
  const int H = a.H;
  const int32_t k0 = beg + sl.ep;
  float t = 0.0f;
  for (int32_t k = k0; k < end; k += 2 * sl.EP) {
    const bool two = k + sl.EP < end;
    const int32_t j0 = a.col[k];
    const int32_t j1 = a.col[two ? k + sl.EP : k];  // unconditional (clamped) load: no join wait
    const VecF<VEC> x0 = ldv<VEC>(a.xh + roff(j0, a.ld_xh) + sl.f0);
    const VecF<VEC> x1 = ldv<VEC>(a.xh + roff(j1, a.ld_xh) + sl.f0);
    const float al0 = a.alpha[roff(k, H) + sl.hs];
    const float al1 = a.alpha[roff(two ? k + sl.EP : k, H) + sl.hs];  // used only when two
    const float z0 = a.a_s[roff(j0, H) + sl.hs] + adr;
    const float z1 = a.a_s[roff(j1, H) + sl.hs] + adr;
    const float da0 = head_sum(vdot<VEC>(x0, dO), sl.L, sl.hfirst) * inv_h;
    const float da1 = head_sum(vdot<VEC>(x1, dO), sl.L, sl.hfirst) * inv_h;
    if (k == k0) {
      q0 = BwdSlot{da0, al0, z0 > 0.0f};
      q1 = BwdSlot{da1, al1, z1 > 0.0f};
    } else if (writer) {
      a.dz[roff(k, H) + sl.hs] = da0;
      if (two) a.dz[roff(k + sl.EP, H) + sl.hs] = da1;
    }
    t += al0 * da0;
    if (two) t += al1 * da1;
  }
  return t;
}

// Writer lanes only: dz = leaky'(z) * alpha * (d alpha - t) per slot, returns their sum.
__device__ __forceinline__ float bwd_pass2(const GatArgs& a, const SlotLane& sl, int32_t beg, int32_t end, float adr,
                                           float t, const BwdSlot& q0, const BwdSlot& q1) {
  const int H = a.H;
  const int32_t k0 = beg + sl.ep;
  float sdz = 0.0f;
  if (k0 < end) {
    const float de = q0.al * (q0.da - t);
    const float v = q0.pos ? de : de * a.slope;
    a.dz[roff(k0, H) + sl.hs] = v;
    sdz += v;
  }
  if (k0 + sl.EP < end) {
    const float de = q1.al * (q1.da - t);
    const float v = q1.pos ? de : de * a.slope;
    a.dz[roff(k0 + sl.EP, H) + sl.hs] = v;
    sdz += v;
  }
#pragma unroll 1
  for (int32_t k = k0 + 2 * sl.EP; k < end; k += sl.EP) {
    const int32_t j = a.col[k];
    float* p = a.dz + roff(k, H) + sl.hs;
    const float de = a.alpha[roff(k, H) + sl.hs] * (*p - t);
    const float v = a.a_s[roff(j, H) + sl.hs] + adr > 0.0f ? de : de * a.slope;
    *p = v;
    sdz += v;
  }
  return sdz;
}

// the lane's slice of the row's upstream gradient (concat: its features; mean: its channels)
template <int VEC>
__device__ __forceinline__ VecF<VEC> load_dO(const GatArgs& a, const SlotLane& sl, int64_t r, bool ok) {
  VecF<VEC> d;
#pragma unroll
  for (int i = 0; i < VEC; ++i) d.v[i] = 0.0f;
  if (a.pdz) {  // dy = dz[r, :] · proj
    if (ok && sl.ok) {
      for (int q = 0; q < a.pnproj; ++q) {
        const float zq = a.pdz[r * a.ld_pdz + q];
        const VecF<VEC> w = ldv<VEC>(a.pproj + (int64_t)q * (a.H * a.C) + sl.f0);
#pragma unroll
        for (int i = 0; i < VEC; ++i) d.v[i] = fmaf(zq, w.v[i], d.v[i]);
      }
    }
  } else if (ok && sl.ok) {
    d = ldv<VEC>(a.dout + r * a.ld_dout + (a.concat ? sl.f0 : sl.c0));
  }
  if (a.y && ok && sl.ok) {  // the store's backward (concat layers), as gat_act_bwd_kernel
    const VecF<VEC> yv = ldv<VEC>(a.y + r * a.ld_y + sl.f0);
    const uint64_t seed = a.pe_seed_ptr ? (*a.pe_seed_ptr) * 0x9E3779B97F4A7C15ull + a.pe_seed : a.pe_seed;
    const int F = a.H * a.C;
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      float g = d.v[i];
      if (a.pe_drop)
        g = keep_elem(seed, (uint32_t)r * (uint32_t)F + (uint32_t)(sl.f0 + i), a.pe_thresh) ? g * a.pe_scale : 0.0f;
      if (a.pe_act == GNN_ACT_ELU && !(yv.v[i] > 0.0f)) g = g * ((a.pe_drop ? yv.v[i] * a.pe_keep : yv.v[i]) + 1.0f);
      d.v[i] = g;
    }
  }
  return d;
}

// the formed d pre of a row slice (one writer per feature slice: the phase-0 lane)
template <int VEC>
__device__ __forceinline__ void store_dpre(const GatArgs& a, const SlotLane& sl, int64_t r, const VecF<VEC>& d) {
  if (a.dpre && sl.ok && sl.ep == 0) stv<VEC>(a.dpre + r * a.ld_dpre + sl.f0, d);
}

// One block, one long row: 256/FLp slot phases; t and d a_dst merged in the wave by xor
// exchanges and across the waves through LDS in a fixed order.
template <int VEC>
__device__ void gat_bwd_long_row(const GatArgs& a, const GatGeom& g, int64_t r, float* sh) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int H = a.H, C = a.C;
  const SlotLane sl = slot_lane(g, tid, 256, lane, VEC, C);
  const bool writer = sl.ok && sl.fl == sl.hs * sl.L;
  const int32_t beg = a.rowptr[r], end = a.rowptr[r + 1];
  const float adr = a.a_d[r * H + sl.hs];
  const float inv_h = a.concat ? 1.0f : 1.0f / (float)H;
  const VecF<VEC> dO = load_dO<VEC>(a, sl, r, true);
  store_dpre<VEC>(a, sl, r, dO);
  BwdSlot q0{0.0f, 0.0f, false}, q1{0.0f, 0.0f, false};
  float t = sl.ok ? bwd_pass1<VEC>(a, sl, beg, end, adr, dO, inv_h, writer, q0, q1) : 0.0f;
  for (int off = 32; off >= g.FLp; off >>= 1) t += __shfl_xor(t, off);
  if (lane < g.FLp) sh[wave * 64 + sl.fl] = t;
  __syncthreads();
  t = ((sh[sl.fl] + sh[64 + sl.fl]) + sh[128 + sl.fl]) + sh[192 + sl.fl];
  float sdz = writer ? bwd_pass2(a, sl, beg, end, adr, t, q0, q1) : 0.0f;
  for (int off = 32; off >= g.FLp; off >>= 1) sdz += __shfl_xor(sdz, off);
  if (lane < g.FLp) sh[256 + wave * 64 + sl.fl] = sdz;
  __syncthreads();
  if (writer && sl.ep == 0)
    a.dad[r * H + sl.hs] = ((sh[256 + sl.fl] + sh[320 + sl.fl]) + sh[384 + sl.fl]) + sh[448 + sl.fl];
}

template <int VEC>
__global__ __launch_bounds__(256) void gat_bwd_rows_group_kernel(GatArgs a, GatGeom g, GatLong lg) {
  __shared__ float sh[512];
  if ((int)blockIdx.x < lg.n) {
    gat_bwd_long_row<VEC>(a, g, lg.rows[blockIdx.x], sh);
    return;
  }
  const int64_t bid = blockIdx.x - lg.n, nblk = gridDim.x - lg.n;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int H = a.H, C = a.C, G = g.G;
  const int lig = lane & (G - 1);
  const int rpw = 64 >> g.lgG;
  const SlotLane sl = slot_lane(g, lig, G, lane, VEC, C);
  const bool writer = sl.ok && sl.fl == sl.hs * sl.L;
  const float inv_h = a.concat ? 1.0f : 1.0f / (float)H;
  const int64_t rpb = 4 * (int64_t)rpw;
  for (int64_t base = bid * rpb; base < a.N; base += nblk * rpb) {
    const int64_t r = gat_row(a, base + wave * rpw + (lane >> g.lgG));
    int32_t beg = 0, end = 0;
    if (r < a.N) { beg = a.rowptr[r]; end = a.rowptr[r + 1]; }
    const VecF<VEC> dO = load_dO<VEC>(a, sl, r, r < a.N);  // issued beside the rowptr loads
    const float adr_ = a.a_d[(r < a.N ? r : 0) * H + sl.hs];
    const float adr = r < a.N ? adr_ : 0.0f;
    const bool own = r < a.N && end - beg <= lg.T;
    if (a.dxh_rowmax && r < a.N && lig == 0 && (r & (GNN_ROWMAX_ROWS - 1)) == 0) a.dxh_rowmax[r / GNN_ROWMAX_ROWS] = 0u;
    if (!own) end = beg;
    if (own) store_dpre<VEC>(a, sl, r, dO);
    BwdSlot q0{0.0f, 0.0f, false}, q1{0.0f, 0.0f, false};
    float t = sl.ok ? bwd_pass1<VEC>(a, sl, beg, end, adr, dO, inv_h, writer, q0, q1) : 0.0f;
    for (int off = G >> 1; off >= g.FLp; off >>= 1) t += __shfl_xor(t, off);
    float sdz = writer ? bwd_pass2(a, sl, beg, end, adr, t, q0, q1) : 0.0f;
    for (int off = G >> 1; off >= g.FLp; off >>= 1) sdz += __shfl_xor(sdz, off);
    if (own && writer && sl.ep == 0) a.dad[r * H + sl.hs] = sdz;
  }
}

// Backward cols pass (CSC, G lanes per source column): d a_src as the pair-view sum of dz,
// the transposed alpha-weighted gather of upstream rows in the slot view, the score-path
// terms, and the attention-vector gradients accumulated in registers across the columns a
// lane visits (one partial per block; gat_att_reduce_kernel finishes them).
template <int VEC>
__global__ __launch_bounds__(256) void gat_bwd_cols_group_kernel(GatArgs a, GatGeom g, float* __restrict__ part) {
  __shared__ float red[2][4][256];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int H = a.H, C = a.C, G = g.G;
  const int F = H * C;
  const int lig = lane & (G - 1);
  const int gbase = lane - lig;
  const int rpw = 64 >> g.lgG;
  const int hl = lig & (H - 1);
  const int fl = lig & (g.FLp - 1);
  const int ep = lig >> g.lgFLp;
  const int EP = G >> g.lgFLp;
  const bool slot_ok = fl < g.FL;
  const int f0 = fl * VEC;
  const int hs = slot_ok ? f0 / C : 0;
  const int c0 = f0 - hs * C;
  const float inv_h = a.concat ? 1.0f : 1.0f / (float)H;
  const int dcol = a.concat ? f0 : c0;
  VecF<VEC> ps, pd, as, ad;
#pragma unroll
  for (int i = 0; i < VEC; ++i) { ps.v[i] = 0.0f; pd.v[i] = 0.0f; }
  if (slot_ok) { as = ldv<VEC>(a.att_s + f0); ad = ldv<VEC>(a.att_d + f0); }
  const int64_t rpb = 4 * (int64_t)rpw;
  for (int64_t base = (int64_t)blockIdx.x * rpb; base < a.N; base += (int64_t)gridDim.x * rpb) {
    const int64_t j = base + wave * rpw + (lane >> g.lgG);
    const bool valid = j < a.N;
    int32_t beg = 0, end = 0;
    if (valid) { beg = a.colptr[j]; end = a.colptr[j + 1]; }
    const int32_t npair = (end - beg) << g.lgH;
    float s = 0.0f;
    for (int32_t idx = lig; idx < npair; idx += G)
      s += a.dz[(int64_t)a.csc2csr[beg + (idx >> g.lgH)] * H + hl];
    for (int off = G >> 1; off >= H; off >>= 1) s += __shfl_xor(s, off);
    const float dash = __shfl(s, gbase + hs);
    VecF<VEC> acc;
#pragma unroll
    for (int i = 0; i < VEC; ++i) acc.v[i] = 0.0f;
    if (slot_ok) {
      for (int32_t k = beg + ep; k < end; k += EP) {
        const int32_t i_ = a.row[k];
        const float al = a.alpha[(int64_t)a.csc2csr[k] * H + hs];
        const VecF<VEC> d = ldv<VEC>(a.dout + (int64_t)i_ * a.ld_dout + dcol);
#pragma unroll
        for (int i = 0; i < VEC; ++i) acc.v[i] += al * d.v[i];
      }
    }
    for (int off = G >> 1; off >= g.FLp; off >>= 1) {
#pragma unroll
      for (int i = 0; i < VEC; ++i) acc.v[i] += __shfl_xor(acc.v[i], off);
    }
    if (valid && slot_ok && ep == 0) {
      const float dadh = a.dad[j * H + hs];
      const VecF<VEC> x = ldv<VEC>(a.xh + j * a.ld_xh + f0);
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        acc.v[i] = acc.v[i] * inv_h + dash * as.v[i] + dadh * ad.v[i];
        ps.v[i] += dash * x.v[i];
        pd.v[i] += dadh * x.v[i];
      }
      stv<VEC>(a.dxh + j * a.ld_dxh + f0, acc);
    }
    if (a.dxh_rowmax) {  // kernel-uniform: max |dxh| over the wave's rpw rows (one row group when
      // rpw <= GNN_ROWMAX_ROWS: the wave's first row is a multiple of rpw), one atomic per wave
      float m = 0.0f;
      if (valid && slot_ok && ep == 0) {
#pragma unroll
        for (int i = 0; i < VEC; ++i) m = fmaxf(m, fabsf(acc.v[i]));
      }
      const int span = rpw <= GNN_ROWMAX_ROWS ? 64 : G;  // lanes whose rows share a group
      for (int off = span >> 1; off >= 1; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
      if (valid && (lane & (span - 1)) == 0) atomicMax(a.dxh_rowmax + j / GNN_ROWMAX_ROWS, __float_as_uint(m));
    }
  }
  // block partial of d att_src / d att_dst: groups of a wave, then the 4 waves through LDS
  for (int off = 32; off >= G; off >>= 1) {
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      ps.v[i] += __shfl_xor(ps.v[i], off);
      pd.v[i] += __shfl_xor(pd.v[i], off);
    }
  }
  if (lane < G && ep == 0 && slot_ok) {
#pragma unroll
    for (int i = 0; i < VEC; ++i) { red[0][wave][f0 + i] = ps.v[i]; red[1][wave][f0 + i] = pd.v[i]; }
  }
  __syncthreads();
  for (int f = threadIdx.x; f < 2 * F; f += blockDim.x) {
    const int w = f >= F;
    const int ff = f - w * F;
    part[((int64_t)blockIdx.x * 2 + w) * F + ff] =
        ((red[w][0][ff] + red[w][1][ff]) + red[w][2][ff]) + red[w][3][ff];
  }
}

// d att (2F outputs) = sum over the cols pass's block partials: one block per output.
__global__ __launch_bounds__(256) void gat_att_reduce_kernel(int F, int nblk, const float* __restrict__ part,
                                                             float* __restrict__ d_att_s, float* __restrict__ d_att_d) {
  __shared__ float wsum[4];
  const int w = blockIdx.x >= (unsigned)F;
  const int f = blockIdx.x - w * F;
  float s = 0.0f;
  for (int b = threadIdx.x; b < nblk; b += blockDim.x) s += part[((int64_t)b * 2 + w) * F + f];
  for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float t = ((wsum[0] + wsum[1]) + wsum[2]) + wsum[3];
    (w ? d_att_d : d_att_s)[f] = t;
  }
}

// Store-side activation / dropout as one in-place pass (the fused forward's fallback for shapes
// outside the lane-group geometry).
__global__ __launch_bounds__(256) void gat_act_fwd_kernel(int64_t N, int32_t Fo, float* __restrict__ out, int64_t ldo,
                                                          GatEpi e) {
  const uint64_t seed = e.dropout ? gat_seed(e) : 0;
  const int64_t total = N * Fo;
  for (int64_t t = blockIdx.x * 256ll + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int64_t r = t / Fo;
    const int c = (int)(t - r * Fo);
    float* q = out + r * ldo + c;
    *q = gat_store_val(e, seed, *q, r, c, Fo);
  }
}

// z = out · projᵀ row by row (the generic geometry's projection; the group kernels do it in their store)
__global__ __launch_bounds__(256) void gat_proj_rows_kernel(int64_t N, int32_t F, const float* __restrict__ out,
                                                            int64_t ldo, const float* __restrict__ proj, int32_t nproj,
                                                            float* __restrict__ z, int64_t ldz) {
  for (int64_t r = blockIdx.x * 256ll + threadIdx.x; r < N; r += (int64_t)gridDim.x * 256) {
    for (int q = 0; q < nproj; ++q) {
      float s = 0.f;
      for (int f = 0; f < F; ++f) s = fmaf(out[r * ldo + f], proj[(int64_t)q * F + f], s);
      z[r * ldz + q] = s;
    }
  }
}

// dy = dz · proj row by row (the generic geometry's dz-form backward)
__global__ __launch_bounds__(256) void gat_dz_proj_kernel(int64_t N, int32_t F, const float* __restrict__ dz,
                                                          int64_t lddz, const float* __restrict__ proj, int32_t nproj,
                                                          float* __restrict__ dy, int64_t lddy) {
  const int64_t total = N * F;
  for (int64_t t = blockIdx.x * 256ll + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int64_t r = t / F;
    const int f = (int)(t - r * F);
    float s = 0.f;
    for (int q = 0; q < nproj; ++q) s = fmaf(dz[r * lddz + q], proj[(int64_t)q * F + f], s);
    dy[r * lddy + f] = s;
  }
}

// d pre = dy * keep / (1-p) * act'(pre), from the stored y = dropout(act(pre)):
// ELU' = 1 for y > 0, else exp(pre) = elu(pre) + 1 with elu(pre) = y * (1-p) for a kept element.
__global__ __launch_bounds__(256) void gat_act_bwd_kernel(int64_t N, int32_t F, GatEpi e, float keep_p,
                                                          const float* __restrict__ y, int64_t ldy,
                                                          const float* dy, int64_t lddy, float* dp, int64_t ldp) {
  const uint64_t seed = e.dropout ? gat_seed(e) : 0;
  const int64_t total = N * F;
  for (int64_t t = blockIdx.x * 256ll + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int64_t r = t / F;
    const int c = (int)(t - r * F);
    float g = dy[r * lddy + c];
    const float yv = y[r * ldy + c];
    if (e.dropout) g = keep_elem(seed, (uint32_t)r * (uint32_t)F + (uint32_t)c, e.keep_thresh) ? g * e.drop_scale : 0.0f;
    if (e.act == GNN_ACT_ELU && !(yv > 0.0f)) g = g * ((e.dropout ? yv * keep_p : yv) + 1.0f);
    dp[r * ldp + c] = g;
  }
}

GatEpi make_epi(int act, float dropout_p, uint64_t seed, const uint64_t* seed_ptr) {
  GatEpi e{};
  e.act = act;
  e.dropout = dropout_p > 0.0f;
  e.keep_thresh = (uint32_t)((1.0 - (double)dropout_p) * 16777216.0);  // as the NT epilogue (gemm_f32.hip)
  e.drop_scale = e.dropout ? (float)(1.0 / (1.0 - (double)dropout_p)) : 1.0f;
  e.seed = seed;
  e.seed_ptr = seed_ptr;
  return e;
}

unsigned elem_blocks(int64_t n) {
  int64_t b = ceil_div(n, 256);
  if (b > 16384) b = 16384;
  return (unsigned)(b > 0 ? b : 1);
}

int ilog2(int v) { int l = 0; while ((1 << l) < v) ++l; return l; }
int pow2ceil(int v) { return 1 << ilog2(v); }

bool vec_ok(const void* p, int64_t ld, int v) {
  return ((uintptr_t)p % (uintptr_t)(4 * v)) == 0 && ld % v == 0;
}

// ---------------------------------------------------------------- the output layer, narrow (round 6)
// GATNet's last conv, GATConv(hidden, C <= 2, heads=1, concat=False) (src/models/gnn.py:67, :75),
// in the slot-parallel narrow form GCN's and SAGE's output layers have (aggregate.hip
// agg_narrow_lds_kernel): a wave owns 64 consecutive rows, one per lane.  Its slots are staged
// through LDS with lanes over SLOTS (neighbour ids, then their xh rows, all in flight together)
// together with each slot's score a_src[j] = <xh[j], att_src> formed on the way; then each lane
// walks its own row's slots in edge order with an online softmax over e = leaky(a_src[j] + a_dst[i])
// (running max m, sum s and accumulator, rescaled when m grows), out = acc / (s + 1e-16) + bias.
// Once a row ends inside a staging window its alpha = exp(e - m) / (s + 1e-16) is written from the
// staged scores (slots of a row that began in an earlier window — a hub in a heavy wave — are
// re-gathered); a_src / a_dst of the row are written beside.  CE: the
// masked weighted cross entropy of the finished logits in the same launch (gnn_masked_ce_f32's
// arithmetic and 256-row partials, dlogits' block column sums beside them), as
// gnn_gcn_out_ce_f32 does for GCN.
struct GatOutArgs {
  const int32_t* rowptr; const int32_t* col;
  int64_t N; int32_t C; float slope;
  const float* xh; int64_t ld_xh;
  const float* att_s; const float* att_d; const float* bias;
  float* a_s; float* a_d; float* alpha;
  float* out; int64_t ldo;
  const int64_t* ce_y; const uint8_t* ce_mask; const float* ce_w; float ce_inv;
  float* ce_dl; int64_t ce_ldd; float* ce_part; float* ce_cs;
};
template <bool CE>
__global__ __launch_bounds__(256) void gat_out_narrow_kernel(GatOutArgs a) {
  // no implicit FMA contraction: the CE and no-CE instances (and the window sizes) must round the
  // softmax sums identically (tests: the fused-CE step bit-identical to the separate one)
#pragma clang fp contract(off)
  // CAP slots staged per wave and window (a wave's 64 rows: ~140 slots on Elliptic); a row that
  // straddles two windows (a hub in a heavy wave) has its alpha re-gathered by all 64 lanes
  constexpr int CAP = 256, LONG = 32;
  __shared__ float sv[4][3 * CAP];  // per wave: xh[j][0], xh[j][1], a_src[j] of the staged slots
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int64_t r0 = ((int64_t)blockIdx.x * 4 + w) * 64;
  const int C = a.C;
  float lg[4] = {0.f, 0.f, 0.f, 0.f};
  int64_t ce_t = -1;
  uint8_t ce_m = 0;
  float ce_w[2] = {0.f, 0.f};
  if constexpr (!CE) {
    if (r0 >= a.N) return;  // wave-uniform; no block barrier below
  }
  if (r0 < a.N) {
    const int64_t r = r0 + lane;
    const bool rok = r < a.N;
    const int64_t rr = rok ? r : r0;
    const int32_t pbeg = a.rowptr[rok ? r : a.N];
    const int32_t pend = a.rowptr[rok ? r + 1 : a.N];
    const int32_t base = __builtin_amdgcn_readfirstlane(a.rowptr[r0]);
    const int32_t wend = __builtin_amdgcn_readfirstlane(a.rowptr[min(r0 + 64, a.N)]);
    // the row's own operands up front (clamped indices): its xh (a_dst), att vectors, bias, CE
    const float as0 = a.att_s[0], as1 = a.att_s[C > 1 ? 1 : 0];
    const float ad0 = a.att_d[0], ad1 = a.att_d[C > 1 ? 1 : 0];
    const float xi0 = a.xh[rr * a.ld_xh], xi1 = a.xh[rr * a.ld_xh + (C > 1 ? 1 : 0)];
    float pb0 = 0.f, pb1 = 0.f;
    if (a.bias) { pb0 = a.bias[0]; pb1 = a.bias[C > 1 ? 1 : 0]; }
    if constexpr (CE) {
      ce_t = a.ce_y[rr];
      ce_m = a.ce_mask[rr];
      ce_w[0] = a.ce_w[0];
      ce_w[1] = a.ce_w[C > 1 ? 1 : 0];
    }
    const float adr = C > 1 ? xi0 * ad0 + xi1 * ad1 : xi0 * ad0;  // (xh_i * att_dst).sum(-1)
    const float asr = C > 1 ? xi0 * as0 + xi1 * as1 : xi0 * as0;
    float m = -INFINITY, s = 0.f, acc0 = 0.f, acc1 = 0.f;
    float* buf = sv[w];
    auto score = [&](int q, float ad) __attribute__((always_inline)) { return leaky(buf[2 * CAP + q] + ad, a.slope); };
    constexpr int W = CAP, NI = W / 64;
    for (int32_t pb = base; pb < wend; pb += W) {
      const int32_t pe = min(pb + W, wend);
      int32_t nn[NI];
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int32_t k = pb + lane + 64 * i;
        nn[i] = a.col[k < pe ? k : pb];
      }
      float x0[NI], x1[NI];
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const float* xr = a.xh + (int64_t)nn[i] * a.ld_xh;
        x0[i] = xr[0];
        x1[i] = xr[C > 1 ? 1 : 0];
      }
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        buf[lane + 64 * i] = x0[i];
        buf[CAP + lane + 64 * i] = C > 1 ? x1[i] : 0.f;
        buf[2 * CAP + lane + 64 * i] = C > 1 ? x0[i] * as0 + x1[i] * as1 : x0[i] * as0;
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes landed
      __builtin_amdgcn_wave_barrier();
      const int32_t lo = max(pbeg, pb), hi0 = min(pend, pe);
      const int32_t hi = min(hi0, lo + LONG);  // a lane walks at most LONG slots of its row per window
      {  // the lane's slots of this window: their max first (independent LDS reads, no branch),
         // one rescale of what earlier windows summed, then the exp-weighted sums in two chains
        float mw = -INFINITY;
        int32_t k = lo;
        for (; k + 1 < hi; k += 2) mw = fmaxf(mw, fmaxf(score(k - pb, adr), score(k + 1 - pb, adr)));
        if (k < hi) mw = fmaxf(mw, score(k - pb, adr));
        const float mn = fmaxf(m, mw);
        if (mn > m) {
          const float sc = m == -INFINITY ? 0.f : fexp(m - mn);
          s *= sc;
          acc0 *= sc;
          acc1 *= sc;
          m = mn;
        }
        float s2 = 0.f, c02 = 0.f, c12 = 0.f;
        for (k = lo; k + 1 < hi; k += 2) {
          const float p = fexp(score(k - pb, adr) - m), p2 = fexp(score(k + 1 - pb, adr) - m);
          s += p;
          acc0 += p * buf[k - pb];
          acc1 += p * buf[CAP + k - pb];
          s2 += p2;
          c02 += p2 * buf[k + 1 - pb];
          c12 += p2 * buf[CAP + k + 1 - pb];
        }
        if (k < hi) {
          const float p = fexp(score(k - pb, adr) - m);
          s += p;
          acc0 += p * buf[k - pb];
          acc1 += p * buf[CAP + k - pb];
        }
        s += s2;
        acc0 += c02;
        acc1 += c12;
      }
      // the rest of each long row: all 64 lanes over its slots (one softmax state per lane, merged
      // by xor butterflies: symmetric, every lane ends with the same state), then into lane L's;
      // a row wholly inside this window gets its alpha written by all lanes right here
      uint64_t longm = __ballot(hi0 - lo > LONG);
      while (longm) {
        const int L = __builtin_ctzll(longm);
        longm &= longm - 1;
        const int32_t s0 = __builtin_amdgcn_readlane(lo, L) + LONG, s1 = __builtin_amdgcn_readlane(hi0, L);
        const float adL = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(adr), L));
        float mw = -INFINITY, sw = 0.f, c0 = 0.f, c1 = 0.f;
        for (int32_t k = s0 + lane; k < s1; k += 64) {
          const float e = score(k - pb, adL);
          const float mn = fmaxf(mw, e);
          const float sc = fexp(mw - mn), p = fexp(e - mn);
          sw = sw * sc + p;
          c0 = c0 * sc + p * buf[k - pb];
          c1 = c1 * sc + p * buf[CAP + k - pb];
          mw = mn;
        }
        for (int o = 32; o >= 1; o >>= 1) {  // merge (m, s, c) pairs
          const float mo = __shfl_xor(mw, o), so = __shfl_xor(sw, o), co0 = __shfl_xor(c0, o), co1 = __shfl_xor(c1, o);
          const float mn = fmaxf(mw, mo);
          const float ea = mw == -INFINITY ? 0.f : fexp(mw - mn), eb = mo == -INFINITY ? 0.f : fexp(mo - mn);
          sw = sw * ea + so * eb;
          c0 = c0 * ea + co0 * eb;
          c1 = c1 * ea + co1 * eb;
          mw = mn;
        }
        if (lane == L) {  // lane L's own state and the wave's
          const float mn = fmaxf(m, mw);
          const float ea = m == -INFINITY ? 0.f : fexp(m - mn), eb = mw == -INFINITY ? 0.f : fexp(mw - mn);
          s = s * ea + sw * eb;
          acc0 = acc0 * ea + c0 * eb;
          acc1 = acc1 * ea + c1 * eb;
          m = mn;
        }
        const int32_t bL = __builtin_amdgcn_readlane(pbeg, L), eL = __builtin_amdgcn_readlane(pend, L);
        if (bL >= pb && eL <= pe) {  // the whole long row in this window: its alpha, by all lanes
          const float mL = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(m), L));
          const float dL = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(s), L)) + 1e-16f;
          const float rL = frcp(dL);
          for (int32_t k = bL + lane; k < eL; k += 64) a.alpha[k] = fexp(score(k - pb, adL) - mL) * rL;
        }
      }
      const bool ends = pend > pb && pend <= pe;
      if (ends && pbeg >= pb && hi0 - lo <= LONG) {  // a short row wholly in this window: its alpha
        const float rd = frcp(s + 1e-16f);
        for (int32_t k = lo; k < hi0; ++k) a.alpha[k] = fexp(score(k - pb, adr) - m) * rd;
      }
      // rows that began in an earlier window and end here: alpha re-gathered by all 64 lanes
      uint64_t strad = __ballot(ends && pbeg < pb);
      while (strad) {
        const int L = __builtin_ctzll(strad);
        strad &= strad - 1;
        const int32_t bL = __builtin_amdgcn_readlane(pbeg, L), eL = __builtin_amdgcn_readlane(pend, L);
        const float adL = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(adr), L));
        const float mL = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(m), L));
        const float dL = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(s), L)) + 1e-16f;
        for (int32_t k = bL + lane; k < eL; k += 64) {
          const float* xr = a.xh + (int64_t)a.col[k] * a.ld_xh;
          const float sj = C > 1 ? xr[0] * as0 + xr[1] * as1 : xr[0] * as0;  // (the staged scores' rounding)
          a.alpha[k] = fexp(leaky(sj + adL, a.slope) - mL) * frcp(dL);
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
    if (rok) {
      const float denom = s + 1e-16f;
      const float o0 = acc0 / denom + pb0, o1 = acc1 / denom + pb1;
      a.a_s[r] = asr;
      a.a_d[r] = adr;
      a.out[r * a.ldo] = o0;
      if (C > 1) a.out[r * a.ldo + 1] = o1;
      lg[0] = o0;
      lg[1] = o1;
    }
  }
  if constexpr (CE) {
    const int64_t r = r0 + lane;
    float l = 0.f;
    float dlv[4] = {0.f, 0.f, 0.f, 0.f};
    if (r < a.N) {  // masked_ce_kernel<C>: loss_r = -w[y]·log_softmax[y], dl = w[y]/n·(softmax - onehot)
      const int64_t tg = ce_t;
      const bool on = ce_m != 0 && tg >= 0 && tg < C;
      const float wt = tg == 0 ? ce_w[0] : ce_w[1];
      l = masked_ce_row<4>(lg, C, tg, on, on ? wt : 0.f, a.ce_inv, a.ce_dl + r * a.ce_ldd, dlv);
    }
    __shared__ float cesh[4];
    for (int o = 32; o > 0; o >>= 1) l += __shfl_xor(l, o);  // train_ops.hip block_sum, same order
    if (lane == 0) cesh[w] = l;
    __syncthreads();
    if (threadIdx.x == 0) {
      float t = 0.f;
      for (int i = 0; i < 4; ++i) t += cesh[i];
      a.ce_part[blockIdx.x] = t;
    }
    if (a.ce_cs) {  // the block's column sums of dl: each wave's rows by its butterfly, the waves in order
      __shared__ float cssh[2][4];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        float v = c < C ? dlv[c] : 0.f;
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if (lane == 0) cssh[c][w] = v;
      }
      __syncthreads();
      if ((int)threadIdx.x < C) {
        float t = 0.f;
        for (int i = 0; i < 4; ++i) t += cssh[threadIdx.x][i];
        a.ce_cs[(int64_t)blockIdx.x * C + threadIdx.x] = t;
      }
    }
  }
}

// Fast-path geometry, or false when the generic one-wave-per-row kernels must run
// (more than 64 slots of VEC floats, or a head mean whose slots per head are not a power of two).
bool gat_geom(int H, int C, int concat, std::initializer_list<std::pair<const void*, int64_t>> ops, GatGeom* g,
              int* vec) {
  const int F = H * C;
  int v = 4;
  for (; v > 1; v >>= 1) {
    if (C % v) continue;
    bool ok = true;
    for (auto& o : ops) ok = ok && (o.first == nullptr || vec_ok(o.first, o.second, v));
    if (ok) break;
  }
  const int FL = F / v, L = C / v;
  if (FL > 64) return false;
  if (!concat && (L & (L - 1))) return false;
  g->FL = FL;
  g->FLp = pow2ceil(FL);
  g->lgFLp = ilog2(g->FLp);
  g->L = L;
  g->lgH = ilog2(H);
  g->G = std::max(std::max(g->FLp, H), 4);
  g->lgG = ilog2(g->G);
  g->Gb = std::min(64, std::max(4, 2 * H));
  g->lgGb = ilog2(g->Gb);
  *vec = v;
  return true;
}

unsigned group_blocks(int64_t N, int G, int64_t cap) {
  int64_t rpb = 4 * (64 / G);
  int64_t b = ceil_div(N, rpb);
  if (b > cap) b = cap;
  return (unsigned)(b > 0 ? b : 1);
}

// The lane-group kernels index rows and slots with 24-bit multiplies (roff).
bool idx24_ok(const gnn_graph* g, int64_t ld_xh, int H) {
  const int64_t lim = (int64_t)1 << 24;
  return g->num_nodes < lim && g->num_slots < lim && ld_xh < lim && H < lim &&
         g->num_nodes * ld_xh < ((int64_t)1 << 32) && g->num_slots * H < ((int64_t)1 << 32);
}

// Degree order of the plan's CSR split (K0b), or null (row order).
const int32_t* csr_order(const gnn_graph* g) {
  const gnn_split* sp = g->csr_split;
  return (sp && sp->order && sp->num_long > 0) ? sp->order : nullptr;
}

// Long-row list of the plan's CSR split (K0b); none when the plan has no split.
GatLong long_rows(const gnn_graph* g) {
  const gnn_split* sp = g->csr_split;
  if (sp && sp->num_long > 0 && sp->long_seg && sp->num_long < (int64_t)1 << 20)
    return GatLong{sp->long_seg, (int32_t)sp->num_long, sp->seg_len};
  return GatLong{nullptr, 0, INT32_MAX};
}

constexpr int64_t kColsBlocks = 2048;  // cols-pass grid cap = number of d att partials

bool pow2_heads(int H) { return H >= 1 && H <= 64 && (H & (H - 1)) == 0; }

unsigned row_blocks(int64_t N) {
  int64_t b = ceil_div(N, 4);
  if (b > ((int64_t)1 << 20)) b = (int64_t)1 << 20;
  return (unsigned)(b > 0 ? b : 1);
}

template <typename C>
void carve_bwd(C& c, int64_t N, int64_t S, int H, int C_, float** dz, float** dad, float** das, float** part) {
  auto p0 = c.template take<float>((size_t)(S > 0 ? S : 1) * H);
  auto p1 = c.template take<float>((size_t)(N > 0 ? N : 1) * H);
  auto p2 = c.template take<float>((size_t)(N > 0 ? N : 1) * H);
  auto p3 = c.template take<float>((size_t)2048 * 2 * H * C_);  // max(kAttBlocks, kColsBlocks)
  if (dz) { *dz = (float*)p0; *dad = (float*)p1; *das = (float*)p2; *part = (float*)p3; }
}

struct SizerAdapter {
  WorkspaceSizer s;
  template <typename T>
  T* take(size_t n) { s.take<T>(n); return nullptr; }
};

}  // namespace
}  // namespace gnnmp

using namespace gnnmp;

extern "C" gnn_status gnn_gat_scores_f32(int64_t N, int32_t H, int32_t C, const float* xh, int64_t ld_xh,
                                         const float* att_src, const float* att_dst, float* a_src,
                                         float* a_dst, gnn_stream_t stream) {
  if (N < 0 || H < 1 || C < 1 || ld_xh < (int64_t)H * C)
    return fail(GNN_ERR_INVALID_ARG, __func__, "bad sizes");
  if (N == 0) return GNN_OK;
  if (!xh || !att_src || !att_dst || !a_src || !a_dst) return fail(GNN_ERR_INVALID_ARG, __func__, "null");
  hipStream_t st = (hipStream_t)stream;
  gat_scores_kernel<<<(unsigned)ceil_div(N * H, 256), 256, 0, st>>>(N, H, C, xh, ld_xh, att_src, att_dst,
                                                                    a_src, a_dst);
  GNN_LAUNCH_CHECK();
  return GNN_OK;
}

extern "C" gnn_status gnn_gat_fwd_f32(const gnn_graph* g, int32_t H, int32_t C, int32_t concat, float slope,
                                      const float* xh, int64_t ld_xh, const float* a_src, const float* a_dst,
                                      const float* bias, float* alpha, float* out, int64_t ldo,
                                      gnn_stream_t stream) {
  if (!g) return fail(GNN_ERR_INVALID_ARG, __func__, "null graph");
  if (!pow2_heads(H)) return fail(GNN_ERR_UNSUPPORTED, __func__, "heads must be a power of two <= 64");
  if (C < 1 || ld_xh < (int64_t)H * C || ldo < (concat ? (int64_t)H * C : C))
    return fail(GNN_ERR_INVALID_ARG, __func__, "bad sizes");
  if (g->num_nodes == 0) return GNN_OK;
  if (!xh || !a_src || !a_dst || !alpha || !out || !g->rowptr || !g->col)
    return fail(GNN_ERR_INVALID_ARG, __func__, "null");
  GatArgs a{};
  a.rowptr = g->rowptr; a.col = g->col; a.N = g->num_nodes;
  a.order = csr_order(g);
  a.H = H; a.C = C; a.concat = concat; a.slope = slope;
  a.xh = xh; a.ld_xh = ld_xh; a.a_s = a_src; a.a_d = a_dst; a.bias = bias;
  a.alpha = alpha; a.out = out; a.ldo = ldo;
  hipStream_t st = (hipStream_t)stream;
  GatGeom gg;
  int vec = 1;
  if (idx24_ok(g, ld_xh, H) && gat_geom(H, C, concat, {{xh, ld_xh}, {out, ldo}}, &gg, &vec)) {
    const GatLong lg = long_rows(g);
    const unsigned nb = group_blocks(a.N, gg.G, (int64_t)1 << 20) + (unsigned)lg.n;
    const GatEpi ep{};
    if (vec == 4) gat_fwd_group_kernel<4, false><<<nb, 256, 0, st>>>(a, gg, lg, ep);
    else if (vec == 2) gat_fwd_group_kernel<2, false><<<nb, 256, 0, st>>>(a, gg, lg, ep);
    else gat_fwd_group_kernel<1, false><<<nb, 256, 0, st>>>(a, gg, lg, ep);
  } else {
    gat_fwd_kernel<<<row_blocks(a.N), 256, 0, st>>>(a);
  }
  GNN_LAUNCH_CHECK();
  return GNN_OK;
}

extern "C" gnn_status gnn_gat_fwd_fused_f32(const gnn_graph* g, const gnn_gat_fwd_params* p, gnn_stream_t stream) {
  if (!g || !p) return fail(GNN_ERR_INVALID_ARG, __func__, "null graph or params");
  const int32_t H = p->heads, C = p->chans, concat = p->concat;
  if (!pow2_heads(H)) return fail(GNN_ERR_UNSUPPORTED, __func__, "heads must be a power of two <= 64");
  if (C < 1 || p->ld_xh < (int64_t)H * C || p->ldo < (concat ? (int64_t)H * C : C))
    return fail(GNN_ERR_INVALID_ARG, __func__, "bad sizes");
  if (p->act != GNN_ACT_NONE && p->act != GNN_ACT_ELU) return fail(GNN_ERR_INVALID_ARG, __func__, "unknown act");
  if (!(p->dropout_p >= 0.0f && p->dropout_p < 1.0f)) return fail(GNN_ERR_INVALID_ARG, __func__, "dropout_p not in [0, 1)");
  if (p->dropout_p > 0.0f && (int64_t)g->num_nodes * (concat ? (int64_t)H * C : (int64_t)C) >= ((int64_t)1 << 32))
    return fail(GNN_ERR_UNSUPPORTED, __func__, "dropout element index (rows x width) must be < 2^32");
  if (g->num_nodes == 0) return GNN_OK;
  if (!p->xh || !p->att_src || !p->att_dst || !p->a_src || !p->a_dst || !p->alpha || !p->out || !g->rowptr || !g->col)
    return fail(GNN_ERR_INVALID_ARG, __func__, "null");
  GatArgs a{};
  a.rowptr = g->rowptr; a.col = g->col; a.N = g->num_nodes;
  a.order = csr_order(g);
  a.H = H; a.C = C; a.concat = concat; a.slope = p->slope;
  a.xh = p->xh; a.ld_xh = p->ld_xh; a.a_s = p->a_src; a.a_d = p->a_dst; a.bias = p->bias;
  a.att_s = p->att_src; a.att_d = p->att_dst;
  a.alpha = p->alpha; a.out = p->out; a.ldo = p->ldo;
  a.ew = p->edge_w;
  GatEpi ep = make_epi(p->act, p->dropout_p, p->seed, p->seed_ptr);
  ep.as_out = p->a_src;
  ep.ad_out = p->a_dst;
  if (p->nproj < 0 || p->nproj > 4 || (p->nproj > 0 && (!concat || !p->proj || !p->z || p->ldz < p->nproj ||
                                                          (reinterpret_cast<uintptr_t>(p->proj) & 15))))
    return fail(GNN_ERR_INVALID_ARG, __func__, "proj: concat, nproj <= 4, proj (16-byte aligned) and z");
  ep.proj = p->proj; ep.nproj = p->nproj; ep.z = p->z; ep.ldz = p->ldz;
  hipStream_t st = (hipStream_t)stream;
  GatGeom gg;
  int vec = 1;
  if (!p->edge_w && idx24_ok(g, p->ld_xh, H) && (p->nproj == 0 || ((H * C) % 4 == 0 && p->nproj <= 2 && H * C <= 256)) &&
      gat_geom(H, C, concat, {{p->xh, p->ld_xh}, {p->out, p->ldo}, {p->att_src, 0}, {p->att_dst, 0}}, &gg, &vec)) {
    const GatLong lg = long_rows(g);
    const unsigned nb = group_blocks(a.N, gg.G, (int64_t)1 << 20) + (unsigned)lg.n;
    if (vec == 4) gat_fwd_group_kernel<4, true><<<nb, 256, 0, st>>>(a, gg, lg, ep);
    else if (vec == 2) gat_fwd_group_kernel<2, true><<<nb, 256, 0, st>>>(a, gg, lg, ep);
    else gat_fwd_group_kernel<1, true><<<nb, 256, 0, st>>>(a, gg, lg, ep);
    GNN_LAUNCH_CHECK();
    return GNN_OK;
  }
  // generic geometry: scores pass, one wave per row, then the activation / dropout pass
  gat_scores_kernel<<<(unsigned)ceil_div(a.N * H, 256), 256, 0, st>>>(a.N, H, C, p->xh, p->ld_xh, p->att_src,
                                                                      p->att_dst, p->a_src, p->a_dst);
  GNN_LAUNCH_CHECK();
  gat_fwd_kernel<<<row_blocks(a.N), 256, 0, st>>>(a);
  GNN_LAUNCH_CHECK();
  if (ep.act != GNN_ACT_NONE || ep.dropout) {
    const int32_t Fo = concat ? H * C : C;
    gat_act_fwd_kernel<<<elem_blocks(a.N * Fo), 256, 0, st>>>(a.N, Fo, p->out, p->ldo, ep);
    GNN_LAUNCH_CHECK();
  }
  if (ep.nproj > 0) {
    gat_proj_rows_kernel<<<elem_blocks(a.N), 256, 0, st>>>(a.N, H * C, p->out, p->ldo, ep.proj, ep.nproj, ep.z, ep.ldz);
    GNN_LAUNCH_CHECK();
  }
  return GNN_OK;
}

extern "C" gnn_status gnn_gat_act_bwd_f32(int64_t N, int64_t F, gnn_act act, float dropout_p, uint64_t seed,
                                          const uint64_t* seed_ptr, const float* y, int64_t ldy, const float* dy,
                                          int64_t lddy, float* dpre, int64_t ld_dpre, gnn_stream_t stream) {
  if (N < 0 || F < 1 || F > INT32_MAX || ldy < F || lddy < F || ld_dpre < F)
    return fail(GNN_ERR_INVALID_ARG, __func__, "bad sizes");
  if (act != GNN_ACT_NONE && act != GNN_ACT_ELU) return fail(GNN_ERR_INVALID_ARG, __func__, "unknown act");
  if (!(dropout_p >= 0.0f && dropout_p < 1.0f)) return fail(GNN_ERR_INVALID_ARG, __func__, "dropout_p not in [0, 1)");
  if (dropout_p > 0.0f && N * F >= ((int64_t)1 << 32)) return fail(GNN_ERR_UNSUPPORTED, __func__, "dropout element index (rows x width) must be < 2^32");
  if (N == 0) return GNN_OK;
  if (!y || !dy || !dpre) return fail(GNN_ERR_INVALID_ARG, __func__, "null");
  const GatEpi ep = make_epi(act, dropout_p, seed, seed_ptr);
  const float keep_p = (float)(1.0 - (double)dropout_p);
  gat_act_bwd_kernel<<<elem_blocks(N * F), 256, 0, (hipStream_t)stream>>>(N, (int32_t)F, ep, keep_p, y, ldy, dy,
                                                                         lddy, dpre, ld_dpre);
  GNN_LAUNCH_CHECK();
  return GNN_OK;
}

namespace gnnmp {
namespace {
// max |x| over each GNN_ROWMAX_ROWS-row group of x [N, F] (float bits, one wave per group): the
// generic kernels' dxh_rowmax (the group kernels form it as they store dxh)
__global__ __launch_bounds__(256) void rowmax_group_kernel(const float* __restrict__ x, int64_t ld, int64_t N, int32_t F,
                                                          uint32_t* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t grp = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int64_t r0 = grp * GNN_ROWMAX_ROWS;
  if (r0 >= N) return;
  const int64_t n = min<int64_t>(GNN_ROWMAX_ROWS, N - r0) * F;
  float m = 0.0f;
  for (int64_t e = lane; e < n; e += 64) m = fmaxf(m, fabsf(x[(r0 + e / F) * ld + e % F]));
  for (int off = 32; off >= 1; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
  if (lane == 0) out[grp] = __float_as_uint(m);
}
}  // namespace
}  // namespace gnnmp

extern "C" gnn_status gnn_gat_bwd_workspace_size(int64_t N, int64_t S, int32_t H, int32_t C, size_t* bytes) {
  if (!bytes || N < 0 || S < 0 || H < 1 || C < 1) return fail(GNN_ERR_INVALID_ARG, __func__, "bad args");
  SizerAdapter a;
  carve_bwd(a, N, S, H, C, nullptr, nullptr, nullptr, nullptr);
  *bytes = a.s.used + 256;
  return GNN_OK;
}

namespace gnnmp {
namespace {
gnn_status gat_bwd_impl(const char* fn, const gnn_graph* g, int32_t H, int32_t C, int32_t concat, float slope,
                        const float* xh, int64_t ld_xh, const float* a_src, const float* a_dst, const float* att_src,
                        const float* att_dst, const float* alpha, const float* dout, int64_t ld_dout, float* dxh,
                        int64_t ld_dxh, float* d_att_src, float* d_att_dst, const float* edge_w, float* d_edge_w,
                        void* workspace, size_t workspace_bytes, gnn_stream_t stream, const GatArgs* post = nullptr) {
  if (!g) return fail(GNN_ERR_INVALID_ARG, fn, "null graph");
  if (!pow2_heads(H)) return fail(GNN_ERR_UNSUPPORTED, fn, "heads must be a power of two <= 64");
  const int64_t F = (int64_t)H * C;
  const bool dzf = post && post->pdz;  // dy given as dz · proj (dout = dz, ld_dout its pitch)
  if (C < 1 || ld_xh < F || ld_dxh < F || (dzf ? ld_dout < post->pnproj : ld_dout < (concat ? F : C)))
    return fail(GNN_ERR_INVALID_ARG, fn, "bad sizes");
  hipStream_t st = (hipStream_t)stream;
  if (g->num_nodes == 0) {
    GNN_HIP_TRY(hipMemsetAsync(d_att_src, 0, F * sizeof(float), st));
    GNN_HIP_TRY(hipMemsetAsync(d_att_dst, 0, F * sizeof(float), st));
    return GNN_OK;
  }
  if (!xh || !a_src || !a_dst || !att_src || !att_dst || !alpha || !dout || !dxh || !d_att_src || !d_att_dst ||
      !g->colptr || !g->row || !g->csc2csr)
    return fail(GNN_ERR_INVALID_ARG, fn, "null");
  WorkspaceCarver c(workspace, workspace_bytes);
  GatArgs a{};
  float* part = nullptr;
  carve_bwd(c, g->num_nodes, g->num_slots, H, C, &a.dz, &a.dad, &a.das, &part);
  if (!c.ok) return fail(GNN_ERR_WORKSPACE, fn, "workspace too small");
  a.rowptr = g->rowptr; a.col = g->col; a.colptr = g->colptr; a.row = g->row; a.csc2csr = g->csc2csr;
  a.order = csr_order(g);
  a.N = g->num_nodes; a.H = H; a.C = C; a.concat = concat; a.slope = slope;
  a.xh = xh; a.ld_xh = ld_xh; a.a_s = a_src; a.a_d = a_dst;
  a.att_s = att_src; a.att_d = att_dst; a.alpha = const_cast<float*>(alpha);
  a.dout = dout; a.ld_dout = ld_dout; a.dxh = dxh; a.ld_dxh = ld_dxh;
  a.ew = edge_w; a.dew = d_edge_w;
  GatGeom gg;
  int vec = 1;
  const bool fuse = post != nullptr;  // the store's backward rides in the rows pass
  const int64_t F_ = (int64_t)H * C;
  if (!edge_w && idx24_ok(g, ld_xh, H) && (!dzf || F % 4 == 0) &&
      gat_geom(H, C, concat, {{xh, ld_xh}, {dzf ? nullptr : dout, dzf ? 0 : ld_dout}, {dxh, ld_dxh}, {att_src, 0}, {att_dst, 0},
                              {fuse ? post->y : nullptr, fuse ? post->ld_y : 0},
                              {fuse ? post->dpre : nullptr, fuse ? post->ld_dpre : 0}}, &gg, &vec)) {
    const GatLong lg = long_rows(g);
    const unsigned nbr = group_blocks(a.N, gg.G, (int64_t)1 << 20) + (unsigned)lg.n;
    const unsigned nbc = group_blocks(a.N, gg.G, kColsBlocks);
    GatArgs ar = a;  // rows pass: dy in, d pre formed and written; cols pass reads d pre
    if (fuse) {
      ar.y = post->y; ar.ld_y = post->ld_y; ar.dpre = post->dpre; ar.ld_dpre = post->ld_dpre;
      ar.pe_act = post->pe_act; ar.pe_drop = post->pe_drop; ar.pe_thresh = post->pe_thresh;
      ar.pe_scale = post->pe_scale; ar.pe_keep = post->pe_keep; ar.pe_seed = post->pe_seed;
      ar.pe_seed_ptr = post->pe_seed_ptr;
      ar.pdz = post->pdz; ar.ld_pdz = post->ld_pdz; ar.pproj = post->pproj; ar.pnproj = post->pnproj;
      a.dout = post->dpre; a.ld_dout = post->ld_dpre;
      ar.dxh_rowmax = a.dxh_rowmax = post->dxh_rowmax;
    }
    switch (vec) {
#define GNN_GAT_BWD(V)                                                            \
  case V:                                                                         \
    gat_bwd_rows_group_kernel<V><<<nbr, 256, 0, st>>>(ar, gg, lg);                \
    GNN_LAUNCH_CHECK();                                                           \
    gat_bwd_cols_group_kernel<V><<<nbc, 256, 0, st>>>(a, gg, part);               \
    break;
      GNN_GAT_BWD(4)
      GNN_GAT_BWD(2)
      default: GNN_GAT_BWD(1)
#undef GNN_GAT_BWD
    }
    GNN_LAUNCH_CHECK();
    gat_att_reduce_kernel<<<(unsigned)(2 * F), 256, 0, st>>>((int)F, (int)nbc, part, d_att_src, d_att_dst);
    GNN_LAUNCH_CHECK();
    return GNN_OK;
  }
  if (fuse && dzf) {  // generic geometry, dz form: dy = dz · proj into dpre first (the act pass below is in place)
    gat_dz_proj_kernel<<<elem_blocks(a.N * F_), 256, 0, st>>>(a.N, (int32_t)F_, post->pdz, post->ld_pdz, post->pproj,
                                                              post->pnproj, post->dpre, post->ld_dpre);
    GNN_LAUNCH_CHECK();
    dout = post->dpre;
    ld_dout = post->ld_dpre;
  }
  if (fuse) {  // generic geometry: the store's backward as its own pass first
    GatEpi ep{};
    ep.act = post->pe_act; ep.dropout = post->pe_drop; ep.keep_thresh = post->pe_thresh; ep.drop_scale = post->pe_scale;
    ep.seed = post->pe_seed; ep.seed_ptr = post->pe_seed_ptr;
    gat_act_bwd_kernel<<<elem_blocks(a.N * F_), 256, 0, st>>>(a.N, (int32_t)F_, ep, post->pe_keep, post->y, post->ld_y,
                                                             dout, ld_dout, post->dpre, post->ld_dpre);
    GNN_LAUNCH_CHECK();
    a.dout = post->dpre; a.ld_dout = post->ld_dpre;
  }
  gat_bwd_rows_kernel<<<row_blocks(a.N), 256, 0, st>>>(a);
  GNN_LAUNCH_CHECK();
  gat_bwd_cols_kernel<<<row_blocks(a.N), 256, 0, st>>>(a);
  GNN_LAUNCH_CHECK();
  if (post && post->dxh_rowmax) {  // the generic kernels: the row-group maxima in a pass of their own
    rowmax_group_kernel<<<(unsigned)ceil_div(ceil_div(a.N, GNN_ROWMAX_ROWS), 4), 256, 0, st>>>(
        dxh, ld_dxh, a.N, (int32_t)F_, post->dxh_rowmax);
    GNN_LAUNCH_CHECK();
  }
  int64_t nblk = a.N < kAttBlocks ? a.N : kAttBlocks;
  int64_t rpb = ceil_div(a.N, nblk);
  nblk = ceil_div(a.N, rpb);
  gat_att_partial_kernel<<<(unsigned)nblk, 256, 0, st>>>(a, rpb, part);
  GNN_LAUNCH_CHECK();
  gat_att_final_kernel<<<(unsigned)ceil_div(F, 256), 256, 0, st>>>((int)F, (int)nblk, part, d_att_src, d_att_dst);
  GNN_LAUNCH_CHECK();
  return GNN_OK;
}
}  // namespace
}  // namespace gnnmp

extern "C" gnn_status gnn_gat_bwd_f32(const gnn_graph* g, int32_t H, int32_t C, int32_t concat, float slope,
                                      const float* xh, int64_t ld_xh, const float* a_src, const float* a_dst,
                                      const float* att_src, const float* att_dst, const float* alpha,
                                      const float* dout, int64_t ld_dout, float* dxh, int64_t ld_dxh,
                                      float* d_att_src, float* d_att_dst, void* workspace,
                                      size_t workspace_bytes, gnn_stream_t stream) {
  return gat_bwd_impl(__func__, g, H, C, concat, slope, xh, ld_xh, a_src, a_dst, att_src, att_dst, alpha, dout,
                      ld_dout, dxh, ld_dxh, d_att_src, d_att_dst, nullptr, nullptr, workspace, workspace_bytes,
                      stream);
}

extern "C" gnn_status gnn_gat_bwd_act_f32(const gnn_graph* g, int32_t H, int32_t C, float slope, const float* xh,
                                          int64_t ld_xh, const float* a_src, const float* a_dst, const float* att_src,
                                          const float* att_dst, const float* alpha, gnn_act act, float dropout_p,
                                          uint64_t seed, const uint64_t* seed_ptr, const float* y, int64_t ld_y,
                                          const float* dy, int64_t ld_dy, float* dpre, int64_t ld_dpre, float* dxh,
                                          int64_t ld_dxh, float* d_att_src, float* d_att_dst, void* workspace,
                                          size_t workspace_bytes, gnn_stream_t stream) {
  const int64_t F = (int64_t)H * C;
  if (act != GNN_ACT_NONE && act != GNN_ACT_ELU) return fail(GNN_ERR_INVALID_ARG, __func__, "unknown act");
  if (!(dropout_p >= 0.0f && dropout_p < 1.0f)) return fail(GNN_ERR_INVALID_ARG, __func__, "dropout_p not in [0, 1)");
  if (!g || (g->num_nodes > 0 && (!y || !dpre)) || ld_y < F || ld_dpre < F)
    return fail(GNN_ERR_INVALID_ARG, __func__, "bad y / dpre");
  if (dropout_p > 0.0f && g->num_nodes * F >= ((int64_t)1 << 32))
    return fail(GNN_ERR_UNSUPPORTED, __func__, "dropout element index (rows x width) must be < 2^32");
  GatArgs post{};
  const GatEpi ep = make_epi(act, dropout_p, seed, seed_ptr);
  post.y = y; post.ld_y = ld_y; post.dpre = dpre; post.ld_dpre = ld_dpre;
  post.pe_act = ep.act; post.pe_drop = ep.dropout; post.pe_thresh = ep.keep_thresh; post.pe_scale = ep.drop_scale;
  post.pe_keep = (float)(1.0 - (double)dropout_p); post.pe_seed = seed; post.pe_seed_ptr = seed_ptr;
  return gat_bwd_impl(__func__, g, H, C, 1, slope, xh, ld_xh, a_src, a_dst, att_src, att_dst, alpha, dy, ld_dy, dxh,
                      ld_dxh, d_att_src, d_att_dst, nullptr, nullptr, workspace, workspace_bytes, stream, &post);
}

extern "C" gnn_status gnn_gat_bwd_act_proj_f32(const gnn_graph* g, int32_t H, int32_t C, float slope, const float* xh,
                                               int64_t ld_xh, const float* a_src, const float* a_dst,
                                               const float* att_src, const float* att_dst, const float* alpha, gnn_act act,
                                               float dropout_p, uint64_t seed, const uint64_t* seed_ptr, const float* y,
                                               int64_t ld_y, const float* dz, int64_t ld_dz, const float* proj,
                                               int32_t nproj, float* dpre, int64_t ld_dpre, float* dxh, int64_t ld_dxh,
                                               float* d_att_src, float* d_att_dst, uint32_t* dxh_rowmax, void* workspace,
                                               size_t workspace_bytes, gnn_stream_t stream) {
  const int64_t F = (int64_t)H * C;
  if (act != GNN_ACT_NONE && act != GNN_ACT_ELU) return fail(GNN_ERR_INVALID_ARG, __func__, "unknown act");
  if (!(dropout_p >= 0.0f && dropout_p < 1.0f)) return fail(GNN_ERR_INVALID_ARG, __func__, "dropout_p not in [0, 1)");
  if (!g || (g->num_nodes > 0 && (!y || !dpre || !dz || !proj)) || ld_y < F || ld_dpre < F || nproj < 1 || nproj > 4 ||
      ld_dz < nproj || (reinterpret_cast<uintptr_t>(proj) & 15))
    return fail(GNN_ERR_INVALID_ARG, __func__, "bad y / dpre / dz / proj");
  if (dropout_p > 0.0f && g->num_nodes * F >= ((int64_t)1 << 32))
    return fail(GNN_ERR_UNSUPPORTED, __func__, "dropout element index (rows x width) must be < 2^32");
  GatArgs post{};
  const GatEpi ep = make_epi(act, dropout_p, seed, seed_ptr);
  post.y = y; post.ld_y = ld_y; post.dpre = dpre; post.ld_dpre = ld_dpre;
  post.pe_act = ep.act; post.pe_drop = ep.dropout; post.pe_thresh = ep.keep_thresh; post.pe_scale = ep.drop_scale;
  post.pe_keep = (float)(1.0 - (double)dropout_p); post.pe_seed = seed; post.pe_seed_ptr = seed_ptr;
  post.pdz = dz; post.ld_pdz = ld_dz; post.pproj = proj; post.pnproj = nproj;
  post.dxh_rowmax = dxh_rowmax;
  return gat_bwd_impl(__func__, g, H, C, 1, slope, xh, ld_xh, a_src, a_dst, att_src, att_dst, alpha, dz, ld_dz, dxh,
                      ld_dxh, d_att_src, d_att_dst, nullptr, nullptr, workspace, workspace_bytes, stream, &post);
}

extern "C" gnn_status gnn_gat_bwd_ew_f32(const gnn_graph* g, int32_t H, int32_t C, int32_t concat, float slope,
                                         const float* xh, int64_t ld_xh, const float* a_src, const float* a_dst,
                                         const float* att_src, const float* att_dst, const float* alpha,
                                         const float* dout, int64_t ld_dout, float* dxh, int64_t ld_dxh,
                                         float* d_att_src, float* d_att_dst, const float* edge_w, float* d_edge_w,
                                         void* workspace, size_t workspace_bytes, gnn_stream_t stream) {
  if (!edge_w || (g && g->num_slots > 0 && !d_edge_w))
    return fail(GNN_ERR_INVALID_ARG, __func__, "edge_w and d_edge_w are required");
  return gat_bwd_impl(__func__, g, H, C, concat, slope, xh, ld_xh, a_src, a_dst, att_src, att_dst, alpha, dout,
                      ld_dout, dxh, ld_dxh, d_att_src, d_att_dst, edge_w, d_edge_w, workspace, workspace_bytes,
                      stream);
}

extern "C" gnn_status gnn_masked_ce_finish(const float* partial, int32_t nblk, float inv_denom, float* loss,
                                           gnn_stream_t stream);

extern "C" gnn_status gnn_gat_out_ce_f32(const gnn_graph* g, const gnn_gat_fwd_params* p, const int64_t* y,
                                         const uint8_t* mask, const float* class_w, float inv_denom, float* dlogits,
                                         int64_t ld_d, float* colsum, float* loss, void* workspace,
                                         size_t workspace_bytes, gnn_stream_t stream) {
  const char* fn = __func__;
  if (!g || !p) return fail(GNN_ERR_INVALID_ARG, fn, "null graph or params");
  if (p->heads != 1 || p->chans < 1 || p->chans > 2 || p->concat || p->act != GNN_ACT_NONE || p->dropout_p != 0.0f ||
      p->edge_w)
    return fail(GNN_ERR_UNSUPPORTED, fn, "the narrow output form: heads 1, 1 <= C <= 2, no concat / act / dropout / edge_w");
  const int64_t N = g->num_nodes;
  if (p->ld_xh < p->chans || p->ldo < p->chans) return fail(GNN_ERR_INVALID_ARG, fn, "bad leading dimensions");
  if (N < 1 || !p->xh || !p->att_src || !p->att_dst || !p->a_src || !p->a_dst || !p->alpha || !p->out || !g->rowptr ||
      (g->num_slots > 0 && !g->col))
    return fail(GNN_ERR_INVALID_ARG, fn, "null operand / N < 1");
  const bool ce = y != nullptr;
  if (ce && (!mask || !class_w || !dlogits || ld_d < p->chans)) return fail(GNN_ERR_INVALID_ARG, fn, "CE operands");
  const int nblk = (int)ceil_div(N, 256);
  if (ce && (!workspace || workspace_bytes < (size_t)nblk * sizeof(float)))
    return fail(GNN_ERR_WORKSPACE, fn, "workspace too small");
  GatOutArgs a{};
  a.rowptr = g->rowptr; a.col = g->col; a.N = N; a.C = p->chans; a.slope = p->slope;
  a.xh = p->xh; a.ld_xh = p->ld_xh; a.att_s = p->att_src; a.att_d = p->att_dst; a.bias = p->bias;
  a.a_s = p->a_src; a.a_d = p->a_dst; a.alpha = p->alpha; a.out = p->out; a.ldo = p->ldo;
  hipStream_t st = (hipStream_t)stream;
  if (!ce) {
    gat_out_narrow_kernel<false><<<(unsigned)nblk, 256, 0, st>>>(a);
    return hip_check(hipGetLastError(), fn);
  }
  a.ce_y = y; a.ce_mask = mask; a.ce_w = class_w; a.ce_inv = inv_denom; a.ce_dl = dlogits; a.ce_ldd = ld_d;
  a.ce_part = static_cast<float*>(workspace); a.ce_cs = colsum;
  gat_out_narrow_kernel<true><<<(unsigned)nblk, 256, 0, st>>>(a);
  const gnn_status s = hip_check(hipGetLastError(), fn);
  if (s != GNN_OK || !loss) return s;  // loss NULL: the partials stay in the workspace (ClipAdam / finish)
  return gnn_masked_ce_finish(static_cast<float*>(workspace), nblk, inv_denom, loss, stream);
}
