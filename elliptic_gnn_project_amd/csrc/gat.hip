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
};

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
        float al = a.alpha[(int64_t)a.csc2csr[k] * H + h];
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
};

__device__ __forceinline__ uint64_t gat_seed(const GatEpi& e) {
  return e.seed_ptr ? (*e.seed_ptr) * 0x9E3779B97F4A7C15ull + e.seed : e.seed;
}

__device__ __forceinline__ float gat_store_val(const GatEpi& e, uint64_t seed, float v, int64_t r, int col, int Fo) {
  if (e.act == GNN_ACT_ELU) v = v > 0.0f ? v : expm1f(v);
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
  __device__ __forceinline__ void add(float e, const VecF<VEC>& x) {
    const float mn = fmaxf(m, e);
    const float sc = expf(m - mn);
    const float p = expf(e - mn);
    s = s * sc + p;
#pragma unroll
    for (int i = 0; i < VEC; ++i) acc.v[i] = acc.v[i] * sc + p * x.v[i];
    m = mn;
  }
  __device__ __forceinline__ void merge(float m2, float s2, const VecF<VEC>& acc2) {
    const float mn = fmaxf(m, m2);
    const float c1 = m == -INFINITY ? 0.0f : expf(m - mn);
    const float c2 = m2 == -INFINITY ? 0.0f : expf(m2 - mn);
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
// the lanes of a head share their trip count, so the head_sum exchanges stay converged).
template <int VEC, bool XS>
__device__ __forceinline__ void slot_pass(const GatArgs& a, const SlotLane& sl, int32_t beg, int32_t end, float adr,
                                          const VecF<VEC>& as_v, bool writer, Online<VEC>& st) {
  const int H = a.H;
  for (int32_t k = beg + sl.ep; k < end; k += 2 * sl.EP) {
    const bool two = k + sl.EP < end;
    const int32_t j0 = a.col[k];
    const int32_t j1 = two ? a.col[k + sl.EP] : j0;
    const VecF<VEC> x0 = ldv<VEC>(a.xh + (int64_t)j0 * a.ld_xh + sl.f0);
    const VecF<VEC> x1 = ldv<VEC>(a.xh + (int64_t)j1 * a.ld_xh + sl.f0);
    float s0, s1;
    if constexpr (XS) {
      s0 = head_sum(vdot<VEC>(x0, as_v), sl.L, sl.hfirst);
      s1 = head_sum(vdot<VEC>(x1, as_v), sl.L, sl.hfirst);
    } else {
      s0 = a.a_s[(int64_t)j0 * H + sl.hs];
      s1 = a.a_s[(int64_t)j1 * H + sl.hs];
    }
    const float e0 = leaky(s0 + adr, a.slope);
    if (writer) a.alpha[(int64_t)k * H + sl.hs] = e0;
    st.add(e0, x0);
    if (two) {
      const float e1 = leaky(s1 + adr, a.slope);
      if (writer) a.alpha[(int64_t)(k + sl.EP) * H + sl.hs] = e1;
      st.add(e1, x1);
    }
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
    if (sl.ok) xr = ldv<VEC>(a.xh + r * a.ld_xh + sl.f0);
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
  if (sl.ok) slot_pass<VEC, XS>(a, sl, beg, end, adr, as_v, writer, st);
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
  const float denom = tot.s + 1e-16f;
  if (a.concat) {
    if (sl.ok && sl.ep == 0) {
      VecF<VEC> o;
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        const int f = sl.f0 + i;
        o.v[i] = gat_store_val(ep_, seed, tot.acc.v[i] / denom + (a.bias ? a.bias[f] : 0.0f), r, f, Fo);
      }
      stv<VEC>(a.out + r * a.ldo + sl.f0, o);
    }
  } else {
    if (sl.ok && sl.ep == 0) {
#pragma unroll
      for (int i = 0; i < VEC; ++i) fin[sl.f0 + i] = tot.acc.v[i] / denom;
    }
    __syncthreads();
    for (int c = tid; c < C; c += 256) {
      float t = 0.0f;
      for (int h = 0; h < H; ++h) t += fin[h * C + c];
      a.out[r * a.ldo + c] = gat_store_val(ep_, seed, t / (float)H + (a.bias ? a.bias[c] : 0.0f), r, c, Fo);
    }
  }
  if (writer) {  // the lane's own raw scores, normalised in place
#pragma unroll 1
    for (int32_t k = beg + sl.ep; k < end; k += sl.EP) {
      float* p = a.alpha + (int64_t)k * H + sl.hs;
      *p = expf(*p - tot.m) / denom;
    }
  }
}

// Forward, short rows (<= T slots): G lanes per row in the slot view, one pass with an online
// softmax per lane, merged across the EP slot phases by xor exchanges; out = acc / (s + 1e-16)
// (+ bias, activation, dropout).  The lane that owns a (head, phase) writes each slot's raw
// score e into alpha during the pass and normalises it afterwards (its own writes, re-read).
// XS: the scores come from the gathered xh rows themselves (a_src[j] = <xh[j,h,:], att_src[h]>,
// reduced over the head's lanes), so the only dependent loads per row are rowptr -> col -> xh.
template <int VEC, bool XS>
__global__ __launch_bounds__(256) void gat_fwd_group_kernel(GatArgs a, GatGeom g, GatLong lg, GatEpi ep_) {
  __shared__ float sh[kLongLds];
  const int lane = threadIdx.x & 63;
  const int H = a.H, C = a.C, F = H * C;
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
    const int64_t r = base + wave * rpw + (lane >> g.lgG);
    int32_t beg = 0, end = 0;
    if (r < a.N) { beg = a.rowptr[r]; end = a.rowptr[r + 1]; }
    const bool own = r < a.N && end - beg <= lg.T;
    if (!own) end = beg;
    float adr;
    if constexpr (XS) {
      VecF<VEC> xr;
#pragma unroll
      for (int i = 0; i < VEC; ++i) xr.v[i] = 0.0f;
      if (own && sl.ok) xr = ldv<VEC>(a.xh + r * a.ld_xh + sl.f0);
      const float ps = head_sum(vdot<VEC>(xr, as_v), sl.L, sl.hfirst);
      adr = head_sum(vdot<VEC>(xr, ad_v), sl.L, sl.hfirst);
      if (own && sl.ep == 0 && writer) {
        ep_.as_out[r * H + sl.hs] = ps;
        ep_.ad_out[r * H + sl.hs] = adr;
      }
    } else {
      adr = own ? a.a_d[r * H + sl.hs] : 0.0f;
    }
    Online<VEC> st;
    st.init();
    if (sl.ok) slot_pass<VEC, XS>(a, sl, beg, end, adr, as_v, writer, st);
    for (int off = G >> 1; off >= g.FLp; off >>= 1) {
      VecF<VEC> a2;
#pragma unroll
      for (int i = 0; i < VEC; ++i) a2.v[i] = __shfl_xor(st.acc.v[i], off);
      st.merge(__shfl_xor(st.m, off), __shfl_xor(st.s, off), a2);
    }
    const float denom = st.s + 1e-16f;
    VecF<VEC> o;
#pragma unroll
    for (int i = 0; i < VEC; ++i) o.v[i] = st.acc.v[i] / denom;
    if (!a.concat) {  // mean over heads: same channel sits L slots apart (L, H powers of two)
      for (int off = g.FLp >> 1; off >= g.L; off >>= 1) {
#pragma unroll
        for (int i = 0; i < VEC; ++i) o.v[i] += __shfl_xor(o.v[i], off);
      }
    }
    if (own && sl.ok && sl.ep == 0) {
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
    if (writer) {
#pragma unroll 1
      for (int32_t k = beg + sl.ep; k < end; k += sl.EP) {
        float* p = a.alpha + (int64_t)k * H + sl.hs;
        *p = expf(*p - st.m) / denom;
      }
    }
  }
}

// Backward rows pass, one long row per block: the same two sweeps as the group kernel below
// with 256 pair lanes and the per-head sums t / d a_dst taken across the waves through LDS.
template <int VEC>
__device__ void gat_bwd_long_row(const GatArgs& a, const GatGeom& g, int64_t r, float* sh) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int H = a.H, C = a.C;
  const int32_t beg = a.rowptr[r], end = a.rowptr[r + 1];
  const int32_t npair = (end - beg) << g.lgH;
  const int hl = tid & (H - 1);
  const float adr = a.a_d[r * H + hl];
  const float inv_h = a.concat ? 1.0f : 1.0f / (float)H;
  const float* dor = a.dout + r * a.ld_dout + (a.concat ? (int64_t)hl * C : 0);
  const float* alpha_r = a.alpha + (int64_t)beg * H;
  float* dz_r = a.dz + (int64_t)beg * H;
  float t = 0.0f;
  for (int32_t idx = tid; idx < npair; idx += 256) {
    const int32_t j = a.col[beg + (idx >> g.lgH)];
    const float* xr = a.xh + (int64_t)j * a.ld_xh + (int64_t)hl * C;
    float da = 0.0f;
    for (int c = 0; c < C; c += VEC) {
      const VecF<VEC> d = ldv<VEC>(dor + c), x = ldv<VEC>(xr + c);
#pragma unroll
      for (int i = 0; i < VEC; ++i) da += d.v[i] * x.v[i];
    }
    da *= inv_h;
    dz_r[idx] = da;
    t += alpha_r[idx] * da;
  }
  for (int off = 32; off >= H; off >>= 1) t += __shfl_xor(t, off);
  if (lane < H) sh[wave * 64 + lane] = t;
  __syncthreads();
  t = ((sh[hl] + sh[64 + hl]) + sh[128 + hl]) + sh[192 + hl];
  float sdz = 0.0f;
  for (int32_t idx = tid; idx < npair; idx += 256) {
    const int32_t j = a.col[beg + (idx >> g.lgH)];
    const float de = alpha_r[idx] * (dz_r[idx] - t);
    const float z = a.a_s[(int64_t)j * H + hl] + adr;
    const float dzv = z > 0.0f ? de : de * a.slope;
    dz_r[idx] = dzv;
    sdz += dzv;
  }
  for (int off = 32; off >= H; off >>= 1) sdz += __shfl_xor(sdz, off);
  if (lane < H) sh[256 + wave * 64 + lane] = sdz;
  __syncthreads();
  if (tid < H) a.dad[r * H + tid] = ((sh[256 + tid] + sh[320 + tid]) + sh[384 + tid]) + sh[448 + tid];
}

// Backward rows pass (pair view, Gb lanes per row): d alpha per (slot, head) as a C-long dot
// of the row's upstream gradient with the neighbour's features, kept in dz between the two
// sweeps; then the softmax and leaky-relu backward and d a_dst = sum over the row.  The first
// pair of each lane keeps its d alpha, alpha and score sign in registers, so a short row's
// second sweep re-reads nothing.
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
  const int H = a.H, C = a.C, G = g.Gb;
  const int lig = lane & (G - 1);
  const int rpw = 64 >> g.lgGb;
  const int hl = lig & (H - 1);
  const float inv_h = a.concat ? 1.0f : 1.0f / (float)H;
  const int64_t rpb = 4 * (int64_t)rpw;
  for (int64_t base = bid * rpb; base < a.N; base += nblk * rpb) {
    const int64_t r = base + wave * rpw + (lane >> g.lgGb);
    int32_t beg = 0, end = 0;
    if (r < a.N) { beg = a.rowptr[r]; end = a.rowptr[r + 1]; }
    const bool own = r < a.N && end - beg <= lg.T;
    if (!own) end = beg;
    const int32_t npair = (end - beg) << g.lgH;
    const float adr = own ? a.a_d[r * H + hl] : 0.0f;
    const float* dor = a.dout + (own ? r : 0) * a.ld_dout + (a.concat ? (int64_t)hl * C : 0);
    const float* alpha_r = a.alpha + (int64_t)beg * H;
    float* dz_r = a.dz + (int64_t)beg * H;
    float t = 0.0f, da0 = 0.0f, al0 = 0.0f;
    bool pos0 = false;
    for (int32_t idx = lig; idx < npair; idx += G) {
      const int32_t j = a.col[beg + (idx >> g.lgH)];
      const float* xr = a.xh + (int64_t)j * a.ld_xh + (int64_t)hl * C;
      float da = 0.0f;
      for (int c = 0; c < C; c += VEC) {
        const VecF<VEC> d = ldv<VEC>(dor + c), x = ldv<VEC>(xr + c);
#pragma unroll
        for (int i = 0; i < VEC; ++i) da += d.v[i] * x.v[i];
      }
      da *= inv_h;
      const float al = alpha_r[idx];
      if (idx == lig) {
        da0 = da;
        al0 = al;
        pos0 = a.a_s[(int64_t)j * H + hl] + adr > 0.0f;
      } else {
        dz_r[idx] = da;
      }
      t += al * da;
    }
    for (int off = G >> 1; off >= H; off >>= 1) t += __shfl_xor(t, off);
    float sdz = 0.0f;
    if (lig < npair) {
      const float de = al0 * (da0 - t);
      const float dzv = pos0 ? de : de * a.slope;
      dz_r[lig] = dzv;
      sdz = dzv;
    }
    for (int32_t idx = lig + G; idx < npair; idx += G) {
      const int32_t j = a.col[beg + (idx >> g.lgH)];
      const float de = alpha_r[idx] * (dz_r[idx] - t);
      const float z = a.a_s[(int64_t)j * H + hl] + adr;
      const float dzv = z > 0.0f ? de : de * a.slope;
      dz_r[idx] = dzv;
      sdz += dzv;
    }
    for (int off = G >> 1; off >= H; off >>= 1) sdz += __shfl_xor(sdz, off);
    if (own && lig < H) a.dad[r * H + lig] = sdz;
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
  a.H = H; a.C = C; a.concat = concat; a.slope = slope;
  a.xh = xh; a.ld_xh = ld_xh; a.a_s = a_src; a.a_d = a_dst; a.bias = bias;
  a.alpha = alpha; a.out = out; a.ldo = ldo;
  hipStream_t st = (hipStream_t)stream;
  GatGeom gg;
  int vec = 1;
  if (gat_geom(H, C, concat, {{xh, ld_xh}, {out, ldo}}, &gg, &vec)) {
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
  if (g->num_nodes == 0) return GNN_OK;
  if (!p->xh || !p->att_src || !p->att_dst || !p->a_src || !p->a_dst || !p->alpha || !p->out || !g->rowptr || !g->col)
    return fail(GNN_ERR_INVALID_ARG, __func__, "null");
  GatArgs a{};
  a.rowptr = g->rowptr; a.col = g->col; a.N = g->num_nodes;
  a.H = H; a.C = C; a.concat = concat; a.slope = p->slope;
  a.xh = p->xh; a.ld_xh = p->ld_xh; a.a_s = p->a_src; a.a_d = p->a_dst; a.bias = p->bias;
  a.att_s = p->att_src; a.att_d = p->att_dst;
  a.alpha = p->alpha; a.out = p->out; a.ldo = p->ldo;
  GatEpi ep = make_epi(p->act, p->dropout_p, p->seed, p->seed_ptr);
  ep.as_out = p->a_src;
  ep.ad_out = p->a_dst;
  hipStream_t st = (hipStream_t)stream;
  GatGeom gg;
  int vec = 1;
  if (gat_geom(H, C, concat, {{p->xh, p->ld_xh}, {p->out, p->ldo}, {p->att_src, 0}, {p->att_dst, 0}}, &gg, &vec)) {
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
  return GNN_OK;
}

extern "C" gnn_status gnn_gat_act_bwd_f32(int64_t N, int64_t F, gnn_act act, float dropout_p, uint64_t seed,
                                          const uint64_t* seed_ptr, const float* y, int64_t ldy, const float* dy,
                                          int64_t lddy, float* dpre, int64_t ld_dpre, gnn_stream_t stream) {
  if (N < 0 || F < 1 || F > INT32_MAX || ldy < F || lddy < F || ld_dpre < F)
    return fail(GNN_ERR_INVALID_ARG, __func__, "bad sizes");
  if (act != GNN_ACT_NONE && act != GNN_ACT_ELU) return fail(GNN_ERR_INVALID_ARG, __func__, "unknown act");
  if (!(dropout_p >= 0.0f && dropout_p < 1.0f)) return fail(GNN_ERR_INVALID_ARG, __func__, "dropout_p not in [0, 1)");
  if (N == 0) return GNN_OK;
  if (!y || !dy || !dpre) return fail(GNN_ERR_INVALID_ARG, __func__, "null");
  const GatEpi ep = make_epi(act, dropout_p, seed, seed_ptr);
  const float keep_p = (float)(1.0 - (double)dropout_p);
  gat_act_bwd_kernel<<<elem_blocks(N * F), 256, 0, (hipStream_t)stream>>>(N, (int32_t)F, ep, keep_p, y, ldy, dy,
                                                                         lddy, dpre, ld_dpre);
  GNN_LAUNCH_CHECK();
  return GNN_OK;
}

extern "C" gnn_status gnn_gat_bwd_workspace_size(int64_t N, int64_t S, int32_t H, int32_t C, size_t* bytes) {
  if (!bytes || N < 0 || S < 0 || H < 1 || C < 1) return fail(GNN_ERR_INVALID_ARG, __func__, "bad args");
  SizerAdapter a;
  carve_bwd(a, N, S, H, C, nullptr, nullptr, nullptr, nullptr);
  *bytes = a.s.used + 256;
  return GNN_OK;
}

extern "C" gnn_status gnn_gat_bwd_f32(const gnn_graph* g, int32_t H, int32_t C, int32_t concat, float slope,
                                      const float* xh, int64_t ld_xh, const float* a_src, const float* a_dst,
                                      const float* att_src, const float* att_dst, const float* alpha,
                                      const float* dout, int64_t ld_dout, float* dxh, int64_t ld_dxh,
                                      float* d_att_src, float* d_att_dst, void* workspace,
                                      size_t workspace_bytes, gnn_stream_t stream) {
  if (!g) return fail(GNN_ERR_INVALID_ARG, __func__, "null graph");
  if (!pow2_heads(H)) return fail(GNN_ERR_UNSUPPORTED, __func__, "heads must be a power of two <= 64");
  const int64_t F = (int64_t)H * C;
  if (C < 1 || ld_xh < F || ld_dxh < F || ld_dout < (concat ? F : C))
    return fail(GNN_ERR_INVALID_ARG, __func__, "bad sizes");
  hipStream_t st = (hipStream_t)stream;
  if (g->num_nodes == 0) {
    GNN_HIP_TRY(hipMemsetAsync(d_att_src, 0, F * sizeof(float), st));
    GNN_HIP_TRY(hipMemsetAsync(d_att_dst, 0, F * sizeof(float), st));
    return GNN_OK;
  }
  if (!xh || !a_src || !a_dst || !att_src || !att_dst || !alpha || !dout || !dxh || !d_att_src || !d_att_dst ||
      !g->colptr || !g->row || !g->csc2csr)
    return fail(GNN_ERR_INVALID_ARG, __func__, "null");
  WorkspaceCarver c(workspace, workspace_bytes);
  GatArgs a{};
  float* part = nullptr;
  carve_bwd(c, g->num_nodes, g->num_slots, H, C, &a.dz, &a.dad, &a.das, &part);
  if (!c.ok) return fail(GNN_ERR_WORKSPACE, __func__, "workspace too small");
  a.rowptr = g->rowptr; a.col = g->col; a.colptr = g->colptr; a.row = g->row; a.csc2csr = g->csc2csr;
  a.N = g->num_nodes; a.H = H; a.C = C; a.concat = concat; a.slope = slope;
  a.xh = xh; a.ld_xh = ld_xh; a.a_s = a_src; a.a_d = a_dst;
  a.att_s = att_src; a.att_d = att_dst; a.alpha = const_cast<float*>(alpha);
  a.dout = dout; a.ld_dout = ld_dout; a.dxh = dxh; a.ld_dxh = ld_dxh;
  GatGeom gg;
  int vec = 1;
  if (gat_geom(H, C, concat, {{xh, ld_xh}, {dout, ld_dout}, {dxh, ld_dxh}, {att_src, 0}, {att_dst, 0}}, &gg,
               &vec)) {
    const GatLong lg = long_rows(g);
    const unsigned nbr = group_blocks(a.N, gg.Gb, (int64_t)1 << 20) + (unsigned)lg.n;
    const unsigned nbc = group_blocks(a.N, gg.G, kColsBlocks);
    switch (vec) {
#define GNN_GAT_BWD(V)                                                            \
  case V:                                                                         \
    gat_bwd_rows_group_kernel<V><<<nbr, 256, 0, st>>>(a, gg, lg);                 \
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
  gat_bwd_rows_kernel<<<row_blocks(a.N), 256, 0, st>>>(a);
  GNN_LAUNCH_CHECK();
  gat_bwd_cols_kernel<<<row_blocks(a.N), 256, 0, st>>>(a);
  GNN_LAUNCH_CHECK();
  int64_t nblk = a.N < kAttBlocks ? a.N : kAttBlocks;
  int64_t rpb = ceil_div(a.N, nblk);
  nblk = ceil_div(a.N, rpb);
  gat_att_partial_kernel<<<(unsigned)nblk, 256, 0, st>>>(a, rpb, part);
  GNN_LAUNCH_CHECK();
  gat_att_final_kernel<<<(unsigned)ceil_div(F, 256), 256, 0, st>>>((int)F, (int)nblk, part, d_att_src, d_att_dst);
  GNN_LAUNCH_CHECK();
  return GNN_OK;
}
