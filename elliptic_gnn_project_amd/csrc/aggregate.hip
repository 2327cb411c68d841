// K1 / K2 / K4 — atomic-free segmented aggregation over a graph plan (fp32).
//
// Replaces PyG 2.5.3 MessagePassing.propagate for:
//   SAGEConv  (aggr='mean'):   x_j = x.index_select(0, ei[0]); scatter(x_j, ei[1], reduce='mean')
//             = zeros.scatter_add_(x_j) / count.clamp(min=1)          (src/models/gnn.py:49,52,187,193)
//   its backward: grad/count then index_add over ei[0]               (the CSC "MEAN_BWD" mode)
//   GCNConv:  message edge_weight * x_j, aggr='add', edge_weight = dinv[j]*dinv[i]  (gnn.py:28,31)
//   GATConv:  message alpha * x_j per head (gnn.py:72,75)
//
// Mapping (CDNA4): lanes stride the F features with VEC-wide (float2/float4) loads so each
// gathered row is read as contiguous 256-1024 B wave-instructions; a lane group walks the
// slots of several consecutive rows flat, keeping 4 neighbour rows in flight (see
// agg_flat_kernel).  Slots are summed in plan order (PyG edge order) with one accumulator
// per feature: no atomics, bitwise reproducible.  Rows with F <= 8 (2-class logits) use a
// group of 8 lanes per row with lanes over slots instead.
#include "gemm_common.hpp"  // keep_elem: the counter-hash dropout shared with the NT epilogue

namespace gnnmp {
namespace {

template <int VEC>
struct VecT;
template <>
struct VecT<1> { using T = float; };
template <>
struct VecT<2> { using T = float2; };
template <>
struct VecT<4> { using T = float4; };

template <int VEC>
__device__ __forceinline__ void vload(const float* p, float (&v)[VEC]) {
  if constexpr (VEC == 4) {
    float4 t = *reinterpret_cast<const float4*>(p);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  } else if constexpr (VEC == 2) {
    float2 t = *reinterpret_cast<const float2*>(p);
    v[0] = t.x; v[1] = t.y;
  } else {
    v[0] = *p;
  }
}

template <int VEC>
__device__ __forceinline__ void vstore(float* p, const float (&v)[VEC]) {
  if constexpr (VEC == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  } else if constexpr (VEC == 2) {
    *reinterpret_cast<float2*>(p) = make_float2(v[0], v[1]);
  } else {
    *p = v[0];
  }
}

// bf16 rows (bf16-storage path): VEC bf16 per lane-chunk widened to f32 / rounded back (RNE).
template <int VEC>
__device__ __forceinline__ void vload_bf(const uint16_t* p, float (&v)[VEC]) {
  if constexpr (VEC == 8) {
    const uint4 t = *reinterpret_cast<const uint4*>(p);
    v[0] = __uint_as_float(t.x << 16); v[1] = __uint_as_float(t.x & 0xffff0000u);
    v[2] = __uint_as_float(t.y << 16); v[3] = __uint_as_float(t.y & 0xffff0000u);
    v[4] = __uint_as_float(t.z << 16); v[5] = __uint_as_float(t.z & 0xffff0000u);
    v[6] = __uint_as_float(t.w << 16); v[7] = __uint_as_float(t.w & 0xffff0000u);
  } else if constexpr (VEC == 4) {
    const uint2 t = *reinterpret_cast<const uint2*>(p);
    v[0] = __uint_as_float(t.x << 16); v[1] = __uint_as_float(t.x & 0xffff0000u);
    v[2] = __uint_as_float(t.y << 16); v[3] = __uint_as_float(t.y & 0xffff0000u);
  } else if constexpr (VEC == 2) {
    const uint32_t t = *reinterpret_cast<const uint32_t*>(p);
    v[0] = __uint_as_float(t << 16); v[1] = __uint_as_float(t & 0xffff0000u);
  } else {
    v[0] = __uint_as_float((uint32_t)p[0] << 16);
  }
}

__device__ __forceinline__ uint16_t to_bf16(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }

template <int VEC>
__device__ __forceinline__ void vstore_bf(uint16_t* p, const float (&v)[VEC]) {
  if constexpr (VEC == 8) {
    *reinterpret_cast<uint4*>(p) = make_uint4((uint32_t)to_bf16(v[0]) | ((uint32_t)to_bf16(v[1]) << 16),
                                              (uint32_t)to_bf16(v[2]) | ((uint32_t)to_bf16(v[3]) << 16),
                                              (uint32_t)to_bf16(v[4]) | ((uint32_t)to_bf16(v[5]) << 16),
                                              (uint32_t)to_bf16(v[6]) | ((uint32_t)to_bf16(v[7]) << 16));
  } else if constexpr (VEC == 4) {
    *reinterpret_cast<uint2*>(p) = make_uint2((uint32_t)to_bf16(v[0]) | ((uint32_t)to_bf16(v[1]) << 16),
                                              (uint32_t)to_bf16(v[2]) | ((uint32_t)to_bf16(v[3]) << 16));
  } else if constexpr (VEC == 2) {
    *reinterpret_cast<uint32_t*>(p) = (uint32_t)to_bf16(v[0]) | ((uint32_t)to_bf16(v[1]) << 16);
  } else {
    p[0] = to_bf16(v[0]);
  }
}

struct AggArgs {
  const int32_t* ptr;    // segment pointer (rowptr or colptr)
  const int32_t* nbr;    // neighbour per slot (col or row)
  const int32_t* wslot;  // EDGE_W + transpose: csc2csr; else null (slot itself)
  const float* nodew;
  const float* ew;
  int32_t heads;
  int32_t chan;          // F / heads
  const float* x; int64_t ldx;
  float* y; int64_t ldy;
  const float* add; int64_t ld_add;
  const float* add2; int64_t ld_add2;  // a second addend, summed after add (ABI 20)
  const float* bias;
  int32_t relu;
  int64_t nrows;
  int32_t F;
  // long-segment split (gnn_split): main pass over truncated segments writes raw partials of
  // long segments to part[piece0[r]]; pieces / combine passes read the full segments
  const int32_t* piece0;   // null: no split
  const int32_t* order;    // split main pass in degree order: position -> row (null: identity)
  float* part;
  const int32_t* fptr;
  const int32_t* fnbr;
  int32_t seg_len;
  // dropout after bias / ReLU (element r·F + f, keep_elem of the NT epilogue)
  int32_t dropout; uint32_t keep_thresh; float drop_scale; uint64_t seed; const int64_t* seed_ptr;
  // split-image output (gnn_sage_mean_fwd_planes): hi / mid / lo bf16 planes at yp + p·yps, row
  // pitch ldy, columns [F, ywidth) zero
  uint16_t* yp; int64_t yps; int32_t ywidth;
  float yscale;  // half-pair store: the image's pre-scale 2^scale_exp (exact), 1 otherwise
  // K1 of the half-pair path: the dropout keep bits of the NEXT GEMM's output rows (the NT that
  // consumes this image, N = kcols <= 128 columns), bit c of kmask[r·4 + c/32] = keep_elem(seed,
  // r·kcols + c), computed here where the gather leaves the VALU idle
  uint32_t* kmask; int32_t kcols;
  // K1 of the half-pair path may also carry the consuming NT's B-image prep (gnn_sage_mean_fwd_h2
  // prep_b): hp.gblocks extra blocks at the front of the grid run ws_prep_h2_cols, one wave per column
  H2Prep hp;
  // K1 of the half-pair path, hub form (gnn_sage_mean_fwd_h2 hub): rows with deg > hub_deg
  // (hubs[0, nhub)) have no slots in the main pass's ptr / nbr; one block each (nhub extra blocks
  // after the prep blocks) walks the full row fptr / fnbr with its 4 waves and writes it
  int32_t nhub; float hub_deg; const int32_t* hubs;
  // ... and optionally balanced main-pass waves: wave k takes rows [wstart[k], wstart[k + 1]) (<= 64)
  const int32_t* wstart;
  // gnn_sage_out_mean_ce_f32: the masked weighted CE of the finished rows (gnn_masked_ce_f32's
  // arithmetic) in the narrow kernel's epilogue: dlogits into ce_dl, per-256-row loss partials
  const int64_t* ce_y; const uint8_t* ce_mask; const float* ce_w; float ce_inv;
  float* ce_dl; int64_t ce_ldd; float* ce_part;
  float* ce_u; int64_t ce_ldu;  // optional: dl / max(deg, 1) per row (the transposed mean's per-slot term)
  float* ce_cs;                 // optional: per-256-row-block column sums of dl, [block][C] (the bias gradient)
};

__device__ __forceinline__ uint64_t agg_seed(const AggArgs& a) {
  return a.seed_ptr ? (uint64_t)(*a.seed_ptr) * 0x9E3779B97F4A7C15ull + a.seed : a.seed;
}

template <int VEC>
__device__ __forceinline__ void agg_dropout(const AggArgs& a, uint64_t seed, int64_t r, int f0, float (&t)[VEC]) {
  if (a.dropout) {
    const uint32_t i0 = (uint32_t)r * (uint32_t)a.F + (uint32_t)f0;
#pragma unroll
    for (int q = 0; q < VEC; ++q) t[q] = keep_elem(seed, i0 + (uint32_t)q, a.keep_thresh) ? t[q] * a.drop_scale : 0.0f;
  }
}

// Per-slot scaled contribution.
template <int MODE, int VEC>
__device__ __forceinline__ void contrib(const AggArgs& a, int32_t n, int32_t r, int64_t slot,
                                        int f0, float (&v)[VEC]) {
  if constexpr (MODE == GNN_AGG_MEAN_BWD) {
    // PyG's grad / count per element (correctly rounded division).  r11 lab: one reciprocal per
    // slot (v · (1/d), <= 1 ulp off) would save 11 of 105 us on the SAGE-graph F = 64 CSC pass.
    float d = fmaxf(a.nodew[n], 1.0f);
#pragma unroll
    for (int q = 0; q < VEC; ++q) v[q] = v[q] / d;
  } else if constexpr (MODE == GNN_AGG_GCN) {
    // PyG's message edge_weight * x_j, rounded, then summed (this file builds with
    // -ffp-contract=off: an FMA with the accumulation would depend on the code path a walk step
    // takes, and PyG rounds the message before the scatter-add)
    const float w = a.nodew[n] * a.nodew[r];
#pragma unroll
    for (int q = 0; q < VEC; ++q) v[q] = w * v[q];
  } else if constexpr (MODE == GNN_AGG_EDGE_W) {
    int64_t ws = a.wslot ? (int64_t)a.wslot[slot] : slot;
    float w = a.ew[ws * a.heads + f0 / a.chan];
#pragma unroll
    for (int q = 0; q < VEC; ++q) v[q] = w * v[q];
  }
}

// contrib with the neighbour's node weight already loaded (wn = nodew[n]): same arithmetic.
// BF (bf16 storage, the result rounded to bf16): MEAN_BWD multiplies by one correctly rounded
// reciprocal per slot (<= 1 f32 ulp from the quotient, far below the bf16 store's rounding) — the
// per-element IEEE division's ~10 VALU ops bound the F = 128 meanᵀ of configs[4]
template <int MODE, int VEC, bool BF = false>
__device__ __forceinline__ void contrib_w(const AggArgs& a, float wn, int32_t r, float (&v)[VEC]) {
  if constexpr (MODE == GNN_AGG_MEAN_BWD && BF) {
    const float rd = 1.0f / fmaxf(wn, 1.0f);
#pragma unroll
    for (int q = 0; q < VEC; ++q) v[q] = v[q] * rd;
  } else if constexpr (MODE == GNN_AGG_MEAN_BWD) {
    const float d = fmaxf(wn, 1.0f);
#pragma unroll
    for (int q = 0; q < VEC; ++q) v[q] = v[q] / d;
  } else if constexpr (MODE == GNN_AGG_GCN) {
    const float w = wn * a.nodew[r];
#pragma unroll
    for (int q = 0; q < VEC; ++q) v[q] = w * v[q];
  }
}

template <int MODE, int VEC>
__device__ __forceinline__ void finish(const AggArgs& a, int64_t r, int f0, float (&acc)[VEC]) {
  if constexpr (MODE == GNN_AGG_MEAN) {
    float d = fmaxf(a.nodew[r], 1.0f);
#pragma unroll
    for (int q = 0; q < VEC; ++q) acc[q] = acc[q] / d;
  }
  if (a.add) {
    float t[VEC];
    vload<VEC>(a.add + r * a.ld_add + f0, t);
#pragma unroll
    for (int q = 0; q < VEC; ++q) acc[q] += t[q];
  }
  if (a.add2) {
    float t[VEC];
    vload<VEC>(a.add2 + r * a.ld_add2 + f0, t);
#pragma unroll
    for (int q = 0; q < VEC; ++q) acc[q] += t[q];
  }
  if (a.bias) {
#pragma unroll
    for (int q = 0; q < VEC; ++q) acc[q] += a.bias[f0 + q];
  }
  if (a.relu) {
#pragma unroll
    for (int q = 0; q < VEC; ++q) acc[q] = fmaxf(acc[q], 0.0f);
  }
  if (a.dropout) agg_dropout<VEC>(a, agg_seed(a), r, f0, acc);
}

// Wide rows (F > 8): flat-slot walk.  A group of LPS lanes (LPS = the power of two that
// covers F/VEC chunks, or 64 with NCH chunks per lane) owns RPG consecutive rows and walks
// their slots U at a time: U neighbour ids, then U·NCH row-chunk loads are all issued before
// any add, regardless of where rows begin and end.  Row boundaries come from rowptrs held in
// the group's lanes (no global load on the flush path); a row is flushed (mean divide,
// root addend, bias, ReLU, store) when the walk passes its end, empty rows included.  Slots
// are added in plan order: each output is the sequential edge-order sum PyG computes.

constexpr int kU = 4;  // slots in flight per group (r11 lab: 8 measured 12-25 % slower on every F = 64 case)

// PF: the next kU neighbour ids are loaded behind this walk step's row loads (one dependent
// round trip per step instead of two).
template <int MODE, int VEC, int LPS, int NCHMAX, bool PF = false>
__device__ __forceinline__ void agg_flat_body(const AggArgs& a, int32_t rpg, uint32_t bid) {
  const int gl = threadIdx.x & (LPS - 1);
  const int gbase = (threadIdx.x & 63) & ~(LPS - 1);
  const int64_t group = ((int64_t)bid * 256 + threadIdx.x) / LPS;
  const int64_t r0 = group * rpg;
  if (r0 >= a.nrows) return;  // group-uniform
  const int nrow = (int)min((int64_t)rpg, a.nrows - r0);
  const int nchunk = a.F / VEC;
  const int nch = (nchunk + LPS - 1) / LPS;
  const int32_t myptr = a.ptr[r0 + min(gl, nrow)];
  // row of this lane's position (degree-ordered split main pass: positions are not rows)
  const int32_t myrow = a.order ? a.order[r0 + min(gl, nrow - 1)] : (int32_t)(r0 + min(gl, nrow - 1));
  float mydeg = 1.0f;
  if constexpr (MODE == GNN_AGG_MEAN) mydeg = a.nodew[myrow];
  const int32_t mypiece = a.piece0 ? a.piece0[myrow] : -1;
  auto ptr_at = [&](int j) { return __shfl(myptr, gbase + j); };
  auto row_at = [&](int j) { return a.order ? __shfl(myrow, gbase + j) : (int32_t)(r0 + j); };

  float acc[NCHMAX][VEC];
#pragma unroll
  for (int i = 0; i < NCHMAX; ++i)
#pragma unroll
    for (int q = 0; q < VEC; ++q) acc[i][q] = 0.0f;

  const uint64_t dseed = a.dropout ? agg_seed(a) : 0;
  auto flush = [&](int j) {
    const int64_t r = row_at(j);
    float d = 1.0f;
    if constexpr (MODE == GNN_AGG_MEAN) d = fmaxf(__shfl(mydeg, gbase + j), 1.0f);
    const int32_t p0 = __shfl(mypiece, gbase + j);
#pragma unroll
    for (int i = 0; i < NCHMAX; ++i) {
      const int c = gl + LPS * i;
      if (i < nch && c < nchunk && p0 >= 0) {  // long row: raw partial of piece 0
        vstore<VEC>(a.part + (int64_t)p0 * a.F + c * VEC, acc[i]);
      } else if (i < nch && c < nchunk) {
        const int f0 = c * VEC;
        float t[VEC];
#pragma unroll
        for (int q = 0; q < VEC; ++q) t[q] = (MODE == GNN_AGG_MEAN) ? acc[i][q] / d : acc[i][q];
        if (a.add) {
          float ad[VEC];
          vload<VEC>(a.add + r * a.ld_add + f0, ad);
#pragma unroll
          for (int q = 0; q < VEC; ++q) t[q] += ad[q];
        }
        if (a.add2) {
          float ad[VEC];
          vload<VEC>(a.add2 + r * a.ld_add2 + f0, ad);
#pragma unroll
          for (int q = 0; q < VEC; ++q) t[q] += ad[q];
        }
        if (a.bias) {
#pragma unroll
          for (int q = 0; q < VEC; ++q) t[q] += a.bias[f0 + q];
        }
        if (a.relu) {
#pragma unroll
          for (int q = 0; q < VEC; ++q) t[q] = fmaxf(t[q], 0.0f);
        }
        if (a.dropout) agg_dropout<VEC>(a, dseed, r, f0, t);
        vstore<VEC>(a.y + r * a.ldy + f0, t);
      }
#pragma unroll
      for (int q = 0; q < VEC; ++q) acc[i][q] = 0.0f;
    }
  };

  const int32_t send = ptr_at(nrow);
  int j = 0;
  int32_t cend = ptr_at(1);
  int32_t crow = row_at(0);
  const int32_t sbeg = ptr_at(0);
  int32_t n[kU];
  if constexpr (PF) {
#pragma unroll
    for (int u = 0; u < kU; ++u) n[u] = a.nbr[sbeg + u < send ? sbeg + u : max(send - 1, sbeg)];
  }
  for (int32_t s = sbeg; s < send; s += kU) {
    if constexpr (!PF) {
#pragma unroll
      for (int u = 0; u < kU; ++u) n[u] = a.nbr[s + u < send ? s + u : s];
    }
    float v[kU][NCHMAX][VEC];
#pragma unroll
    for (int u = 0; u < kU; ++u)
#pragma unroll
      for (int i = 0; i < NCHMAX; ++i)
        if (i < nch) {
          const int c = gl + LPS * i;
          vload<VEC>(a.x + (int64_t)n[u] * a.ldx + (c < nchunk ? c : 0) * VEC, v[u][i]);
        }
    int32_t nn[kU];
    if constexpr (PF) {
#pragma unroll
      for (int u = 0; u < kU; ++u) nn[u] = a.nbr[min(s + kU + u, send - 1)];
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int32_t k = s + u;
      if (k >= send) break;
      while (k >= cend) {  // passing one or more row ends (empty rows flush zeros)
        flush(j);
        ++j;
        cend = ptr_at(j + 1);
        crow = row_at(j);
      }
#pragma unroll
      for (int i = 0; i < NCHMAX; ++i)
        if (i < nch) {
          contrib<MODE, VEC>(a, n[u], crow, k, (gl + LPS * i) * VEC, v[u][i]);
#pragma unroll
          for (int q = 0; q < VEC; ++q) acc[i][q] += v[u][i][q];
        }
    }
    if constexpr (PF) {
#pragma unroll
      for (int u = 0; u < kU; ++u) n[u] = nn[u];
    }
  }
  for (; j < nrow; ++j) flush(j);  // the last open row and any trailing empty rows
}

// The standalone launch keeps its own copy of the walk (agg_flat_body below is the same code for
// the pieces-folded launch): routed through the device function, hipcc scheduled the 32-lane
// F = 128 pass differently and it measured 11 % slower (r17: 1473 -> 1641 us, scaled config).
template <int MODE, int VEC, int LPS, int NCHMAX, bool PF = false>
__global__ __launch_bounds__(256) void agg_flat_kernel(AggArgs a, int32_t rpg) {
  const int gl = threadIdx.x & (LPS - 1);
  const int gbase = (threadIdx.x & 63) & ~(LPS - 1);
  const int64_t group = ((int64_t)blockIdx.x * 256 + threadIdx.x) / LPS;
  const int64_t r0 = group * rpg;
  if (r0 >= a.nrows) return;  // group-uniform
  const int nrow = (int)min((int64_t)rpg, a.nrows - r0);
  const int nchunk = a.F / VEC;
  const int nch = (nchunk + LPS - 1) / LPS;
  const int32_t myptr = a.ptr[r0 + min(gl, nrow)];
  // row of this lane's position (degree-ordered split main pass: positions are not rows)
  const int32_t myrow = a.order ? a.order[r0 + min(gl, nrow - 1)] : (int32_t)(r0 + min(gl, nrow - 1));
  float mydeg = 1.0f;
  if constexpr (MODE == GNN_AGG_MEAN) mydeg = a.nodew[myrow];
  const int32_t mypiece = a.piece0 ? a.piece0[myrow] : -1;
  auto ptr_at = [&](int j) { return __shfl(myptr, gbase + j); };
  auto row_at = [&](int j) { return a.order ? __shfl(myrow, gbase + j) : (int32_t)(r0 + j); };

  float acc[NCHMAX][VEC];
#pragma unroll
  for (int i = 0; i < NCHMAX; ++i)
#pragma unroll
    for (int q = 0; q < VEC; ++q) acc[i][q] = 0.0f;

  const uint64_t dseed = a.dropout ? agg_seed(a) : 0;
  auto flush = [&](int j) {
    const int64_t r = row_at(j);
    float d = 1.0f;
    if constexpr (MODE == GNN_AGG_MEAN) d = fmaxf(__shfl(mydeg, gbase + j), 1.0f);
    const int32_t p0 = __shfl(mypiece, gbase + j);
#pragma unroll
    for (int i = 0; i < NCHMAX; ++i) {
      const int c = gl + LPS * i;
      if (i < nch && c < nchunk && p0 >= 0) {  // long row: raw partial of piece 0
        vstore<VEC>(a.part + (int64_t)p0 * a.F + c * VEC, acc[i]);
      } else if (i < nch && c < nchunk) {
        const int f0 = c * VEC;
        float t[VEC];
#pragma unroll
        for (int q = 0; q < VEC; ++q) t[q] = (MODE == GNN_AGG_MEAN) ? acc[i][q] / d : acc[i][q];
        if (a.add) {
          float ad[VEC];
          vload<VEC>(a.add + r * a.ld_add + f0, ad);
#pragma unroll
          for (int q = 0; q < VEC; ++q) t[q] += ad[q];
        }
        if (a.add2) {
          float ad[VEC];
          vload<VEC>(a.add2 + r * a.ld_add2 + f0, ad);
#pragma unroll
          for (int q = 0; q < VEC; ++q) t[q] += ad[q];
        }
        if (a.bias) {
#pragma unroll
          for (int q = 0; q < VEC; ++q) t[q] += a.bias[f0 + q];
        }
        if (a.relu) {
#pragma unroll
          for (int q = 0; q < VEC; ++q) t[q] = fmaxf(t[q], 0.0f);
        }
        if (a.dropout) agg_dropout<VEC>(a, dseed, r, f0, t);
        vstore<VEC>(a.y + r * a.ldy + f0, t);
      }
#pragma unroll
      for (int q = 0; q < VEC; ++q) acc[i][q] = 0.0f;
    }
  };

  const int32_t send = ptr_at(nrow);
  int j = 0;
  int32_t cend = ptr_at(1);
  int32_t crow = row_at(0);
  const int32_t sbeg = ptr_at(0);
  int32_t n[kU];
  if constexpr (PF) {
#pragma unroll
    for (int u = 0; u < kU; ++u) n[u] = a.nbr[sbeg + u < send ? sbeg + u : max(send - 1, sbeg)];
  }
  for (int32_t s = sbeg; s < send; s += kU) {
    if constexpr (!PF) {
#pragma unroll
      for (int u = 0; u < kU; ++u) n[u] = a.nbr[s + u < send ? s + u : s];
    }
    float v[kU][NCHMAX][VEC];
#pragma unroll
    for (int u = 0; u < kU; ++u)
#pragma unroll
      for (int i = 0; i < NCHMAX; ++i)
        if (i < nch) {
          const int c = gl + LPS * i;
          vload<VEC>(a.x + (int64_t)n[u] * a.ldx + (c < nchunk ? c : 0) * VEC, v[u][i]);
        }
    int32_t nn[kU];
    if constexpr (PF) {
#pragma unroll
      for (int u = 0; u < kU; ++u) nn[u] = a.nbr[min(s + kU + u, send - 1)];
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int32_t k = s + u;
      if (k >= send) break;
      while (k >= cend) {  // passing one or more row ends (empty rows flush zeros)
        flush(j);
        ++j;
        cend = ptr_at(j + 1);
        crow = row_at(j);
      }
#pragma unroll
      for (int i = 0; i < NCHMAX; ++i)
        if (i < nch) {
          contrib<MODE, VEC>(a, n[u], crow, k, (gl + LPS * i) * VEC, v[u][i]);
#pragma unroll
          for (int q = 0; q < VEC; ++q) acc[i][q] += v[u][i][q];
        }
    }
    if constexpr (PF) {
#pragma unroll
      for (int u = 0; u < kU; ++u) n[u] = nn[u];
    }
  }
  for (; j < nrow; ++j) flush(j);  // the last open row and any trailing empty rows
}

// Wave-wide groups (LPS = 64, F/VEC > 32 chunks, e.g. the 166-wide layer-1 features):
// every row boundary and neighbour id is wave-uniform, so they live in SGPRs (scalar loads,
// v_readlane) and the next U neighbour ids are prefetched while the current U rows load.
// PLN: y is written as a split image, no split partials: 3 = split-bf16 planes (hi / mid / lo
// bf16), 2 = half-pair planes (hi / lo f16, gemm_common.hpp split_h2_pair); VEC even.
// One hub row of K1's half-pair store, by a whole block: wave w sums the row's slot groups
// w, w + 4, w + 8, ... (U slots each, in slot order, the next group's ids loaded behind the
// current rows), then wave 0 adds waves 1..3 in order, divides by max(deg, 1) and writes the
// half-pair planes (zero padding columns) as agg_wave_kernel's flush does.  A strong-scaling
// shard's degree-196 row walked by one wave was its K1's tail (profiles/r47_shards.txt).
template <int VEC, int NCH>
__device__ __forceinline__ void k1_hub_row(const AggArgs& a, int32_t r) {
  constexpr int U = 8, W = 4;
  __shared__ float red[(W - 1) * NCH * VEC * 64];  // [wave - 1][chunk][q][lane]: conflict-free
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int32_t beg = a.fptr[r], end = a.fptr[r + 1];  // end > beg: deg > hub_deg >= 1
  const int nchunk = a.F / VEC;
  int coff[NCH];
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c = lane + 64 * i;
    coff[i] = (c < nchunk ? c : 0) * VEC;
  }
  float acc[NCH][VEC];
#pragma unroll
  for (int i = 0; i < NCH; ++i)
#pragma unroll
    for (int q = 0; q < VEC; ++q) acc[i][q] = 0.0f;
  int32_t n[U];
#pragma unroll
  for (int u = 0; u < U; ++u) n[u] = __builtin_amdgcn_readfirstlane(a.fnbr[min(beg + w * U + u, end - 1)]);
  for (int32_t s = beg + w * U; s < end; s += W * U) {
    float v[U][NCH][VEC];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int i = 0; i < NCH; ++i) vload<VEC>(a.x + (int64_t)n[u] * a.ldx + coff[i], v[u][i]);
#pragma unroll
    for (int u = 0; u < U; ++u) n[u] = __builtin_amdgcn_readfirstlane(a.fnbr[min(s + W * U + u, end - 1)]);
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (s + u < end) {
#pragma unroll
        for (int i = 0; i < NCH; ++i)
#pragma unroll
          for (int q = 0; q < VEC; ++q) acc[i][q] += v[u][i][q];
      }
  }
  if (w > 0) {
#pragma unroll
    for (int i = 0; i < NCH; ++i)
#pragma unroll
      for (int q = 0; q < VEC; ++q) red[(((w - 1) * NCH + i) * VEC + q) * 64 + lane] = acc[i][q];
  }
  __syncthreads();
  if (w != 0) return;
#pragma unroll
  for (int ww = 0; ww < W - 1; ++ww)
#pragma unroll
    for (int i = 0; i < NCH; ++i)
#pragma unroll
      for (int q = 0; q < VEC; ++q) acc[i][q] += red[((ww * NCH + i) * VEC + q) * 64 + lane];
  const float d = fmaxf(a.nodew[r], 1.0f);
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c = lane + 64 * i;
    if (!(c < nchunk || c * VEC < a.ywidth)) continue;
    uint32_t wd[VEC / 2][2];
#pragma unroll
    for (int q = 0; q < VEC / 2; ++q) {
      const float t0 = c < nchunk ? acc[i][2 * q] / d : 0.0f;
      const float t1 = c < nchunk ? acc[i][2 * q + 1] / d : 0.0f;
      split_h2_pair(t0 * a.yscale, t1 * a.yscale, wd[q][0], wd[q][1]);
    }
    uint16_t* dst = a.yp + (int64_t)r * a.ldy + c * VEC;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      if constexpr (VEC == 4) *reinterpret_cast<uint2*>(dst + p * a.yps) = make_uint2(wd[0][p], wd[1][p]);
      else *reinterpret_cast<uint32_t*>(dst + p * a.yps) = wd[0][p];
    }
  }
}

template <int MODE, int VEC, int NCH, bool BF = false, int U = 8, int PLN = 0>  // BF: x and y hold bf16 (no split partials)
__global__ __launch_bounds__(256) void agg_wave_kernel(AggArgs a, int32_t rpg) {
  if constexpr (PLN == 2) {  // the NT's B prep rides along (blocks [0, hp.gblocks), launched first)
    if ((int)blockIdx.x < a.hp.gblocks) {
      ws_prep_h2_cols<256>(a.hp, (int)blockIdx.x);
      return;
    }
    if ((int)blockIdx.x < a.hp.gblocks + a.nhub) {  // the hub rows, also launched early
      k1_hub_row<VEC, NCH>(a, a.hubs[(int)blockIdx.x - a.hp.gblocks]);
      return;
    }
  }
  const int lane = threadIdx.x & 63;
  const int64_t bid = (int64_t)blockIdx.x - (PLN == 2 ? a.hp.gblocks + a.nhub : 0);
  const int64_t wave = (bid * 256 + threadIdx.x) >> 6;
  int64_t r0 = wave * rpg;
  int nrow;
  if (PLN == 2 && a.wstart) {  // balanced waves (rpg = the wave count)
    if (wave >= rpg) return;
    r0 = __builtin_amdgcn_readfirstlane(a.wstart[wave]);
    nrow = __builtin_amdgcn_readfirstlane(a.wstart[wave + 1]) - (int)r0;
    if (nrow <= 0) return;
  } else {
    if (r0 >= a.nrows) return;
    nrow = (int)min((int64_t)rpg, a.nrows - r0);
  }
  const int nchunk = a.F / VEC;
  const int32_t myptr = a.ptr[r0 + min(lane, nrow)];
  const int32_t myrow = a.order ? a.order[r0 + min(lane, nrow - 1)] : (int32_t)(r0 + min(lane, nrow - 1));
  float mydeg = 1.0f;
  if constexpr (MODE == GNN_AGG_MEAN) mydeg = a.nodew[myrow];
  const int32_t mypiece = a.piece0 ? a.piece0[myrow] : -1;
  auto row_at = [&](int j) { return a.order ? __builtin_amdgcn_readlane(myrow, j) : (int32_t)(r0 + j); };
  int coff[NCH];
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c = lane + 64 * i;
    coff[i] = (c < nchunk ? c : 0) * VEC;
  }
  float acc[NCH][VEC];
#pragma unroll
  for (int i = 0; i < NCH; ++i)
#pragma unroll
    for (int q = 0; q < VEC; ++q) acc[i][q] = 0.0f;

  const uint64_t dseed = a.dropout ? agg_seed(a) : 0;
  auto flush = [&](int j) {
    const int64_t r = row_at(j);
    float d = 1.0f;
    if constexpr (MODE == GNN_AGG_MEAN) d = fmaxf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(mydeg), j)), 1.0f);
    const int32_t p0 = __builtin_amdgcn_readlane(mypiece, j);
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = lane + 64 * i;
      if constexpr (PLN != 0) {
        static_assert(VEC % 2 == 0, "planes are written in column pairs");
        if ((PLN != 2 || !(d > a.hub_deg) || a.nhub == 0) && (c < nchunk || c * VEC < a.ywidth)) {  // (hub rows: k1_hub_row)
          uint32_t w[VEC / 2][3];
#pragma unroll
          for (int q = 0; q < VEC / 2; ++q) {
            const float t0 = c < nchunk ? acc[i][2 * q] / d : 0.0f;
            const float t1 = c < nchunk ? acc[i][2 * q + 1] / d : 0.0f;
            if constexpr (PLN == 3) split3_pair(t0, t1, w[q][0], w[q][1], w[q][2]);
            else split_h2_pair(t0 * a.yscale, t1 * a.yscale, w[q][0], w[q][1]);  // PyG's mean, then 2^exp
          }
          uint16_t* dst = a.yp + r * a.ldy + c * VEC;
#pragma unroll
          for (int p = 0; p < PLN; ++p) {
            if constexpr (VEC == 4) *reinterpret_cast<uint2*>(dst + p * a.yps) = make_uint2(w[0][p], w[1][p]);
            else *reinterpret_cast<uint32_t*>(dst + p * a.yps) = w[0][p];
          }
        }
#pragma unroll
        for (int q = 0; q < VEC; ++q) acc[i][q] = 0.0f;
        if (i == NCH - 1 && a.kmask) {  // once per row, after its planes
          const uint32_t e0 = (uint32_t)r * (uint32_t)a.kcols;
          const bool k0 = lane < a.kcols && keep_elem(dseed, e0 + (uint32_t)lane, a.keep_thresh);
          const bool k1 = lane + 64 < a.kcols && keep_elem(dseed, e0 + (uint32_t)(lane + 64), a.keep_thresh);
          const uint64_t b0 = __ballot(k0), b1 = __ballot(k1);
          if (lane == 0)
            *reinterpret_cast<uint4*>(a.kmask + r * 4) =
                make_uint4((uint32_t)b0, (uint32_t)(b0 >> 32), (uint32_t)b1, (uint32_t)(b1 >> 32));
        }
        continue;
      }
      if (!BF && c < nchunk && p0 >= 0) {  // long row: raw partial of piece 0
        vstore<VEC>(a.part + (int64_t)p0 * a.F + c * VEC, acc[i]);
      } else if (c < nchunk) {
        const int f0 = c * VEC;
        float t[VEC];
#pragma unroll
        for (int q = 0; q < VEC; ++q) t[q] = (MODE == GNN_AGG_MEAN) ? acc[i][q] / d : acc[i][q];
        if (a.add) {
          float ad[VEC];
          vload<VEC>(a.add + r * a.ld_add + f0, ad);
#pragma unroll
          for (int q = 0; q < VEC; ++q) t[q] += ad[q];
        }
        if (a.add2) {
          float ad[VEC];
          vload<VEC>(a.add2 + r * a.ld_add2 + f0, ad);
#pragma unroll
          for (int q = 0; q < VEC; ++q) t[q] += ad[q];
        }
        if (a.bias) {
#pragma unroll
          for (int q = 0; q < VEC; ++q) t[q] += a.bias[f0 + q];
        }
        if (a.relu) {
#pragma unroll
          for (int q = 0; q < VEC; ++q) t[q] = fmaxf(t[q], 0.0f);
        }
        if (a.dropout) agg_dropout<VEC>(a, dseed, r, f0, t);
        if constexpr (BF) vstore_bf<VEC>(reinterpret_cast<uint16_t*>(a.y) + r * a.ldy + f0, t);
        else vstore<VEC>(a.y + r * a.ldy + f0, t);
      }
#pragma unroll
      for (int q = 0; q < VEC; ++q) acc[i][q] = 0.0f;
    }
  };

  const int32_t sbeg = __builtin_amdgcn_readlane(myptr, 0);
  const int32_t send = __builtin_amdgcn_readlane(myptr, nrow);
  int j = 0;
  int32_t cend = __builtin_amdgcn_readlane(myptr, 1);
  int32_t crow = row_at(0);
  int32_t n[U];
#pragma unroll
  for (int u = 0; u < U; ++u) n[u] = __builtin_amdgcn_readfirstlane(a.nbr[min(sbeg + u, max(send - 1, sbeg))]);
  // the per-slot node weight (MEAN_BWD: the neighbour's in-degree; GCN: its D^-1/2) of the U
  // neighbours in flight, loaded one iteration ahead with their ids (a load at the first use
  // waited a scalar round trip per iteration: the bf16 F = 128 meanᵀ ran at 1.9 TB/s)
  constexpr bool SW = MODE == GNN_AGG_MEAN_BWD || MODE == GNN_AGG_GCN;
  const uint32_t nmax = (uint32_t)max<int64_t>(a.nrows - 1, 0);
  float dn[U];
#pragma unroll
  for (int u = 0; u < U; ++u) dn[u] = SW ? a.nodew[min((uint32_t)n[u], nmax)] : 1.0f;
  for (int32_t s = sbeg; s < send; s += U) {
    float v[U][NCH][VEC];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        if constexpr (BF) vload_bf<VEC>(reinterpret_cast<const uint16_t*>(a.x) + (int64_t)n[u] * a.ldx + coff[i], v[u][i]);
        else vload<VEC>(a.x + (int64_t)n[u] * a.ldx + coff[i], v[u][i]);
      }
    int32_t nn[U];  // prefetch the next U neighbour ids behind this iteration's row loads
#pragma unroll
    for (int u = 0; u < U; ++u) nn[u] = __builtin_amdgcn_readfirstlane(a.nbr[min(s + U + u, send - 1)]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int32_t k = s + u;
      if (k >= send) break;
      while (k >= cend) {
        flush(j);
        ++j;
        cend = __builtin_amdgcn_readlane(myptr, j + 1);
        crow = row_at(j);
      }
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        if constexpr (SW) contrib_w<MODE, VEC, BF>(a, dn[u], crow, v[u][i]);
        else contrib<MODE, VEC>(a, n[u], crow, k, coff[i], v[u][i]);
#pragma unroll
        for (int q = 0; q < VEC; ++q) acc[i][q] += v[u][i][q];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      n[u] = nn[u];
      if constexpr (SW) dn[u] = a.nodew[min((uint32_t)n[u], nmax)];
    }
  }
  for (; j < nrow; ++j) flush(j);
}

// bf16 rows of at most 64 / G lane chunks (configs[4]'s F = 128 mean and meanᵀ: 32 chunks of 4 or
// 16 of 8 bf16): the wave's G lane groups gather G consecutive slots per load instruction — group g
// takes slot k + g — so every lane loads (the one-slot agg_wave_kernel leaves 64 − F/VEC lanes idle,
// 32 of 64 at F = 128).  A group adds its own slots in plan order into its own accumulators; a row's
// flush adds the groups' partials by a fixed xor tree over the groups (deterministic, but no longer
// PyG's single sequential chain: the bf16 path stores the sum rounded to bf16 and its tests bound
// it in bf16 ulps).  Neighbour ids and weights stay wave-uniform (scalar); a group selects its
// slot's.  Modes SUM / MEAN / MEAN_BWD (their slot term needs no per-row weight).
template <int MODE, int VEC, int G, int U = 8>
__global__ __launch_bounds__(256) void agg_wave_group_bf16_kernel(AggArgs a, int32_t rpg) {
  static_assert(MODE == GNN_AGG_SUM || MODE == GNN_AGG_MEAN || MODE == GNN_AGG_MEAN_BWD, "no per-row slot weight");
  static_assert(G == 2 || G == 4, "2 or 4 lane groups");
  constexpr int LG = 64 / G;  // lanes per group
  constexpr int S = G * U;    // slots per walk step
  const int lane = threadIdx.x & 63;
  const int grp = lane / LG;
  const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int64_t r0 = wave * rpg;
  if (r0 >= a.nrows) return;
  const int nrow = (int)min((int64_t)rpg, a.nrows - r0);
  const int nchunk = a.F / VEC;
  const int32_t myptr = a.ptr[r0 + min(lane, nrow)];
  float mydeg = 1.0f;
  if constexpr (MODE == GNN_AGG_MEAN) mydeg = a.nodew[r0 + min(lane, nrow - 1)];
  const int c = lane % LG;
  const int coff = (c < nchunk ? c : 0) * VEC;
  const uint16_t* xb = reinterpret_cast<const uint16_t*>(a.x) + coff;
  float acc[VEC];
#pragma unroll
  for (int q = 0; q < VEC; ++q) acc[q] = 0.0f;
  const uint64_t dseed = a.dropout ? agg_seed(a) : 0;
  auto flush = [&](int j) {
    float t[VEC];
#pragma unroll
    for (int q = 0; q < VEC; ++q) {
      t[q] = acc[q] + __shfl_xor(acc[q], LG);                // groups (0 + 1), (2 + 3)
      if constexpr (G == 4) t[q] = t[q] + __shfl_xor(t[q], 2 * LG);  // then (0 + 1) + (2 + 3)
      acc[q] = 0.0f;
    }
    if (grp == 0 && c < nchunk) {
      const int64_t r = r0 + j;
      const int f0 = c * VEC;
      if constexpr (MODE == GNN_AGG_MEAN) {
        const float d = fmaxf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(mydeg), j)), 1.0f);
#pragma unroll
        for (int q = 0; q < VEC; ++q) t[q] = t[q] / d;
      }
      if (a.add) {
#pragma unroll
        for (int q = 0; q < VEC; ++q) t[q] += a.add[r * a.ld_add + f0 + q];
      }
      if (a.bias) {
#pragma unroll
        for (int q = 0; q < VEC; ++q) t[q] += a.bias[f0 + q];
      }
      if (a.relu) {
#pragma unroll
        for (int q = 0; q < VEC; ++q) t[q] = fmaxf(t[q], 0.0f);
      }
      if (a.dropout) agg_dropout<VEC>(a, dseed, r, f0, t);
      vstore_bf<VEC>(reinterpret_cast<uint16_t*>(a.y) + r * a.ldy + f0, t);
    }
  };

  const int32_t sbeg = __builtin_amdgcn_readlane(myptr, 0);
  const int32_t send = __builtin_amdgcn_readlane(myptr, nrow);
  int j = 0;
  int32_t cend = __builtin_amdgcn_readlane(myptr, 1);
  constexpr bool SW = MODE == GNN_AGG_MEAN_BWD;
  const uint32_t nmax = (uint32_t)max<int64_t>(a.nrows - 1, 0);
  int32_t n[S];
#pragma unroll
  for (int u = 0; u < S; ++u) n[u] = __builtin_amdgcn_readfirstlane(a.nbr[min(sbeg + u, max(send - 1, sbeg))]);
  // this lane group's slot of each group of G: oid[m] = n[G·m + grp]; MEAN_BWD: the in-degree of
  // that neighbour (U per lane, not G·U wave-uniform values), loaded one step ahead with the ids
  int32_t oid[U];
  float dn[U];
#pragma unroll
  for (int m = 0; m < U; ++m) {
    oid[m] = n[G * m];
#pragma unroll
    for (int g = 1; g < G; ++g) oid[m] = grp == g ? n[G * m + g] : oid[m];
    dn[m] = SW ? a.nodew[min((uint32_t)oid[m], nmax)] : 1.0f;
  }
  for (int32_t s = sbeg; s < send; s += S) {
    float v[U][VEC];
#pragma unroll
    for (int m = 0; m < U; ++m) vload_bf<VEC>(xb + (int64_t)oid[m] * a.ldx, v[m]);
    int32_t nn[S];  // the next step's ids, behind this step's row loads
#pragma unroll
    for (int u = 0; u < S; ++u) nn[u] = __builtin_amdgcn_readfirstlane(a.nbr[min(s + S + u, send - 1)]);
#pragma unroll
    for (int m = 0; m < U; ++m) {
      if constexpr (SW) contrib_w<MODE, VEC, true>(a, dn[m], 0, v[m]);  // the lane's own slot's term, once
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const int32_t k = s + G * m + g;
        if (k >= send) break;  // wave-uniform
        while (k >= cend) {
          flush(j);
          ++j;
          cend = __builtin_amdgcn_readlane(myptr, j + 1);
        }
        const bool mine = grp == g;
#pragma unroll
        for (int q = 0; q < VEC; ++q) acc[q] = mine ? acc[q] + v[m][q] : acc[q];
      }
    }
#pragma unroll
    for (int m = 0; m < U; ++m) {
      oid[m] = nn[G * m];
#pragma unroll
      for (int g = 1; g < G; ++g) oid[m] = grp == g ? nn[G * m + g] : oid[m];
      if constexpr (SW) dn[m] = a.nodew[min((uint32_t)oid[m], nmax)];
    }
  }
  for (; j < nrow; ++j) flush(j);
}

// Narrow rows (F <= 8, e.g. 2-class logits): a group of 8 lanes per row, lanes over the
// row's slots (hubs are shared by 8 lanes), then a 3-step xor-shuffle reduction.
// NF: compile-time bound on F (2, 4 or 8): every row value is loaded unconditionally (clamped
// index), so a slot's loads issue together instead of one per feature behind its own branch.
constexpr int kGroup = 8;
template <int MODE, int NF>
__global__ __launch_bounds__(256) void agg_group_kernel(AggArgs a) {
  const int sub = threadIdx.x & (kGroup - 1);
  for (int64_t r = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / kGroup; r < a.nrows;
       r += (int64_t)gridDim.x * blockDim.x / kGroup) {
    const int32_t beg = a.ptr[r];
    const int32_t end = a.ptr[r + 1];
    float acc[8];
#pragma unroll
    for (int f = 0; f < 8; ++f) acc[f] = 0.0f;
    const float wr = MODE == GNN_AGG_GCN ? a.nodew[r] : 1.0f;  // the row's weight, once
    for (int32_t k = beg + sub; k < end; k += kGroup) {
      const int32_t n = a.nbr[k];
      const float* xr = a.x + (int64_t)n * a.ldx;
      float xv[NF];
#pragma unroll
      for (int f = 0; f < NF; ++f) xv[f] = xr[f < a.F ? f : 0];
      // the slot's weight loaded beside its row values (contrib's arithmetic, same rounding)
      const float wn = (MODE == GNN_AGG_GCN || MODE == GNN_AGG_MEAN_BWD) ? a.nodew[n] : 1.0f;
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        float v = xv[f];
        if constexpr (MODE == GNN_AGG_GCN) {
          v = (wn * wr) * v;
        } else if constexpr (MODE == GNN_AGG_MEAN_BWD) {
          v = v / fmaxf(wn, 1.0f);
        } else {
          float t[1] = {v};
          contrib<MODE, 1>(a, n, (int32_t)r, k, f, t);
          v = t[0];
        }
        acc[f] += f < a.F ? v : 0.0f;
      }
    }
#pragma unroll
    for (int f = 0; f < NF; ++f) {
#pragma unroll
      for (int off = kGroup / 2; off >= 1; off >>= 1) acc[f] += __shfl_xor(acc[f], off);
    }
    if (sub == 0) {
      // epilogue operands loaded together (clamped indices) — finish<MODE, 1>'s arithmetic
      const int32_t p0 = a.piece0 ? a.piece0[r] : -1;
      const float dr = MODE == GNN_AGG_MEAN ? fmaxf(a.nodew[r], 1.0f) : 1.0f;
      float addv[NF], add2v[NF], bv[NF];
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        const int fc = f < a.F ? f : 0;
        addv[f] = a.add ? a.add[r * a.ld_add + fc] : 0.0f;
        add2v[f] = a.add2 ? a.add2[r * a.ld_add2 + fc] : 0.0f;
        bv[f] = a.bias ? a.bias[fc] : 0.0f;
      }
      const uint64_t dseed = a.dropout ? agg_seed(a) : 0;
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        if (f < a.F) {
          float t[1] = {acc[f]};
          if (p0 >= 0) {
            a.part[(int64_t)p0 * a.F + f] = t[0];
          } else {
            if constexpr (MODE == GNN_AGG_MEAN) t[0] = t[0] / dr;
            if (a.add) t[0] += addv[f];
            if (a.add2) t[0] += add2v[f];
            if (a.bias) t[0] += bv[f];
            if (a.relu) t[0] = fmaxf(t[0], 0.0f);
            if (a.dropout) agg_dropout<1>(a, dseed, r, f, t);
            a.y[r * a.ldy + f] = t[0];
          }
        }
      }
    }
  }
}

// Narrow rows, slot-parallel (F <= 4; MEAN / MEAN_BWD / SUM): a wave owns 64 consecutive rows
// (one per lane).  Their slots are staged through LDS with lanes over SLOTS — neighbour ids
// and the F-wide neighbour rows of 64 slots per instruction, all in flight together — and then
// each lane adds its own row's slots from LDS in edge order (sequential, deterministic; COOP: a
// row's slots past the first 32 of a pass are summed by all 64 lanes, strided, in a fixed xor tree).
// NF (2 or 4): compile-time bound on F.  The staging is branch-free: all neighbour ids of the
// pass, then all their row values (clamped feature index) and weights, then the LDS writes — a
// per-feature `f < F` branch had compiled to one dependent load + vmcnt(0) per value (r10: 16 us
// warm, 21 us cold for ~11 MB).
// CE (gnn_sage_out_mean_ce_f32): each finished row's masked weighted cross entropy in the
// epilogue (masked_ce_kernel's arithmetic, bit for bit: a block's 4 waves x 64 rows are that
// kernel's 256-row block, its loss partial summed in the same order); waves past the last row
// then stay for the block's one barrier instead of returning.
template <int MODE, int NF, int kNarrowCap = 256, bool COOP = false, bool CE = false>  // kNarrowCap: slots staged per pass per wave
__global__ __launch_bounds__(256) void agg_narrow_lds_kernel(AggArgs a) {
  __shared__ float sv[4][kNarrowCap * 4];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int64_t r0 = ((int64_t)blockIdx.x * 4 + w) * 64;
  float lg[4] = {0.f, 0.f, 0.f, 0.f};  // CE: the row's logits
  int64_t ce_t = -1;                   // CE: its label, mask byte and the class weights (prefetched)
  float ce_deg = 1.0f;                 // CE: max(deg, 1) of the row (the u output's divisor)
  uint8_t ce_m = 0;
  float ce_w[4] = {0.f, 0.f, 0.f, 0.f};
  if constexpr (!CE) {
    if (r0 >= a.nrows) return;  // wave-uniform; no block barriers below
  }
  if (r0 < a.nrows) {  // (CE: the block's barrier follows)
  const int64_t r = r0 + lane;
  const bool rok = r < a.nrows;
  const int32_t pbeg = a.ptr[rok ? r : a.nrows];
  const int32_t pend = a.ptr[rok ? r + 1 : a.nrows];
  const int32_t base = __builtin_amdgcn_readfirstlane(a.ptr[r0]);
  const int64_t rlast = min(r0 + 64, a.nrows);
  const int32_t wend = __builtin_amdgcn_readfirstlane(a.ptr[rlast]);
  const int F = a.F;
  // the row's epilogue operands (1/deg, root addend, bias) are loaded up front, in flight with
  // the gather instead of one more dependent round trip after it
  // (clamped row / feature indices, no per-value branch: the epilogue reads only f < F)
  const int64_t rr = rok ? r : r0;
  float pdeg = 1.0f, padd[4] = {0.f, 0.f, 0.f, 0.f}, padd2[4] = {0.f, 0.f, 0.f, 0.f}, pbias[4] = {0.f, 0.f, 0.f, 0.f};
  if constexpr (MODE == GNN_AGG_MEAN) pdeg = fmaxf(a.nodew[rr], 1.0f);
  // GCN (F <= 2): the row's D^-1/2; each slot's message is (dinv_j · dinv_i) · x_j as in
  // agg_group_kernel / contrib (the product of the two weights first, PyG's edge_weight), dinv_j
  // staged in the LDS plane f = 2
  static_assert(MODE != GNN_AGG_GCN || NF == 2, "GCN rows stage their slot weight in plane 2");
  float wrow = 1.0f;
  if constexpr (MODE == GNN_AGG_GCN) wrow = a.nodew[rr];
  if (a.add) {
#pragma unroll
    for (int f = 0; f < NF; ++f) padd[f] = a.add[rr * a.ld_add + (f < F ? f : 0)];
  }
  if (a.add2) {
#pragma unroll
    for (int f = 0; f < NF; ++f) padd2[f] = a.add2[rr * a.ld_add2 + (f < F ? f : 0)];
  }
  if (a.bias) {
#pragma unroll
    for (int f = 0; f < NF; ++f) pbias[f] = a.bias[f < F ? f : 0];
  }
  if constexpr (CE) {  // the CE's row operands too (label, mask, the C class weights): no round trip after the sum
    ce_deg = pdeg;
    ce_t = a.ce_y[rr];
    ce_m = a.ce_mask[rr];
#pragma unroll
    for (int c = 0; c < 4; ++c) ce_w[c] = a.ce_w[c < F ? c : 0];
  }
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  float* buf = sv[w];
  for (int32_t pb = base; pb < wend; pb += kNarrowCap) {
    const int32_t pe = min(pb + kNarrowCap, wend);
    constexpr int NI = kNarrowCap / 64;
    int32_t nn[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int32_t k = pb + lane + 64 * i;
      nn[i] = a.nbr[k < pe ? k : pb];
    }
    float xv[NI][NF], dd[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const float* xr = a.x + (int64_t)nn[i] * a.ldx;
#pragma unroll
      for (int f = 0; f < NF; ++f) xv[i][f] = xr[f < F ? f : 0];
      dd[i] = 1.0f;
      if constexpr (MODE == GNN_AGG_MEAN_BWD || MODE == GNN_AGG_GCN) dd[i] = a.nodew[nn[i]];
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) {
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        float v = f < F ? xv[i][f] : 0.0f;
        if constexpr (MODE == GNN_AGG_MEAN_BWD) v = v / fmaxf(dd[i], 1.0f);
        buf[f * kNarrowCap + lane + 64 * i] = v;
      }
      if constexpr (MODE == GNN_AGG_GCN) buf[2 * kNarrowCap + lane + 64 * i] = dd[i];
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes landed
    __builtin_amdgcn_wave_barrier();
    const int32_t lo = max(pbeg, pb), hi0 = min(pend, pe);
    constexpr int CAP = 32;  // COOP: a lane walks at most CAP slots of its row per pass
    const int32_t hi = COOP ? min(hi0, lo + CAP) : hi0;
    // 4 interleaved partial sums: a hub lane's LDS reads pipeline instead of chaining
    float q1[4] = {0.f, 0.f, 0.f, 0.f}, q2[4] = {0.f, 0.f, 0.f, 0.f}, q3[4] = {0.f, 0.f, 0.f, 0.f};
    // a slot's staged value (GCN: its message, weighted here by the reading row's dinv)
    auto sv_at = [&](int f, int32_t s, float wr) __attribute__((always_inline)) {
      const float x = buf[f * kNarrowCap + (s - pb)];
      if constexpr (MODE == GNN_AGG_GCN) return (buf[2 * kNarrowCap + (s - pb)] * wr) * x;
      else return x;
    };
    int32_t k = lo;
    for (; k + 3 < hi; k += 4) {
#pragma unroll
      for (int f = 0; f < NF; ++f) {  // (features past NF are never staged: NF = 2 reads half)
        acc[f] += sv_at(f, k, wrow);
        q1[f] += sv_at(f, k + 1, wrow);
        q2[f] += sv_at(f, k + 2, wrow);
        q3[f] += sv_at(f, k + 3, wrow);
      }
    }
    for (; k < hi; ++k) {
#pragma unroll
      for (int f = 0; f < NF; ++f) acc[f] += sv_at(f, k, wrow);
    }
#pragma unroll
    for (int f = 0; f < NF; ++f) acc[f] += (q1[f] + q2[f]) + q3[f];
    if constexpr (COOP) {  // the rest of each long row: all 64 lanes, strided, then a fixed xor tree
      uint64_t longm = __ballot(hi0 - lo > CAP);
      while (longm) {
        const int L = __builtin_ctzll(longm);
        longm &= longm - 1;
        const int32_t s0 = __builtin_amdgcn_readlane(lo, L) + CAP, s1 = __builtin_amdgcn_readlane(hi0, L);
        const float wL = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wrow), L));
        float part[NF];
#pragma unroll
        for (int f = 0; f < NF; ++f) part[f] = 0.f;
        for (int32_t k2 = s0 + lane; k2 < s1; k2 += 64) {
#pragma unroll
          for (int f = 0; f < NF; ++f) part[f] += sv_at(f, k2, wL);
        }
#pragma unroll
        for (int f = 0; f < NF; ++f) {
#pragma unroll
          for (int off = 32; off >= 1; off >>= 1) part[f] += __shfl_xor(part[f], off);
          if (lane == L) acc[f] += part[f];
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  if (rok) {
    const int32_t p0 = a.piece0 ? a.piece0[r] : -1;
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      if (f < F) {
        float t[1] = {acc[f]};
        if (p0 >= 0) {
          a.part[(int64_t)p0 * F + f] = t[0];
        } else {  // finish<MODE, 1> with the preloaded operands (same operation order)
          if constexpr (MODE == GNN_AGG_MEAN) t[0] = t[0] / pdeg;
          if (a.add) t[0] += padd[f];
          if (a.add2) t[0] += padd2[f];
          if (a.bias) t[0] += pbias[f];
          if (a.relu) t[0] = fmaxf(t[0], 0.0f);
          if (a.dropout) agg_dropout<1>(a, agg_seed(a), r, f, t);
          a.y[r * a.ldy + f] = t[0];
          lg[f] = t[0];
        }
      }
    }
  }
  }  // r0 < nrows
  if constexpr (CE) {
    const int64_t r = r0 + lane;
    const int C = a.F;
    float l = 0.f;
    float dlv[4] = {0.f, 0.f, 0.f, 0.f};
    if (r < a.nrows) {  // masked_ce_kernel<C>: loss_r = -w[y]·log_softmax[y], dl = w[y]/n·(softmax - onehot)
      const int64_t tg = ce_t;
      const bool on = ce_m != 0 && tg >= 0 && tg < C;
      const float wt = tg == 0 ? ce_w[0] : tg == 1 ? ce_w[1] : tg == 2 ? ce_w[2] : ce_w[3];
      l = masked_ce_row<4>(lg, C, tg, on, on ? wt : 0.f, a.ce_inv, a.ce_dl + r * a.ce_ldd, dlv);
      if (a.ce_u) {  // MEAN_BWD's v / max(deg, 1) of this row, the same division (deg is MEAN's nodew)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (c < C) a.ce_u[r * a.ce_ldu + c] = dlv[c] / ce_deg;
      }
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
      __shared__ float cssh[4][4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
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

// ---- long-segment split: pieces 1.. of every long segment, then the ordered combine.
// Wide rows: one wave per piece, lanes over features, U neighbour rows in flight.
template <int MODE, int VEC, int NCH>
__device__ __forceinline__ void agg_piece_wide_body(const AggArgs& a, int64_t npieces, const int32_t* piece_seg,
                                                    uint32_t bid) {
  constexpr int U = 8;
  const int lane = threadIdx.x & 63;
  const int64_t p = ((int64_t)bid * 256 + threadIdx.x) >> 6;
  if (p >= npieces) return;
  const int32_t r = piece_seg[p];
  const int32_t k = (int32_t)p - a.piece0[r];
  if (k == 0) return;  // piece 0 belongs to the main pass
  const int32_t beg = a.fptr[r] + k * a.seg_len;
  const int32_t end = min(beg + a.seg_len, a.fptr[r + 1]);
  const int nchunk = a.F / VEC;
  float acc[NCH][VEC];
#pragma unroll
  for (int i = 0; i < NCH; ++i)
#pragma unroll
    for (int q = 0; q < VEC; ++q) acc[i][q] = 0.0f;
  for (int32_t s = beg; s < end; s += U) {
    int32_t n[U];
#pragma unroll
    for (int u = 0; u < U; ++u) n[u] = __builtin_amdgcn_readfirstlane(a.fnbr[min(s + u, end - 1)]);
    float v[U][NCH][VEC];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        const int c = lane + 64 * i;
        vload<VEC>(a.x + (int64_t)n[u] * a.ldx + (c < nchunk ? c : 0) * VEC, v[u][i]);
      }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (s + u >= end) break;
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        contrib<MODE, VEC>(a, n[u], r, s + u, (lane + 64 * i) * VEC, v[u][i]);
#pragma unroll
        for (int q = 0; q < VEC; ++q) acc[i][q] += v[u][i][q];
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c = lane + 64 * i;
    if (c < nchunk) vstore<VEC>(a.part + p * a.F + c * VEC, acc[i]);
  }
}

template <int MODE, int VEC, int NCH>
__global__ __launch_bounds__(256) void agg_piece_wide_kernel(AggArgs a, int64_t npieces, const int32_t* piece_seg) {
  agg_piece_wide_body<MODE, VEC, NCH>(a, npieces, piece_seg, blockIdx.x);
}

// The split main pass and the split pieces in ONE launch: blocks [0, pblocks) walk the long
// segments' pieces (one wave each, launched first so the hubs start early), the rest the
// degree-ordered main pass; both only write (partials / rows), the combine pass follows.
template <int MODE, int VEC, int LPS, int NCHMAX>
__global__ __launch_bounds__(256) void agg_flat_pieces_kernel(AggArgs a, int32_t rpg, int64_t npieces,
                                                              const int32_t* piece_seg, uint32_t pblocks) {
  if (blockIdx.x < pblocks) agg_piece_wide_body<MODE, VEC, 1>(a, npieces, piece_seg, blockIdx.x);
  else agg_flat_body<MODE, VEC, LPS, NCHMAX>(a, rpg, blockIdx.x - pblocks);
}

// Narrow rows (F <= 8): one wave per piece, lanes over its <= 64 slots, fixed xor tree.
template <int MODE>
__global__ __launch_bounds__(256) void agg_piece_narrow_kernel(AggArgs a, int64_t npieces, const int32_t* piece_seg) {
  const int lane = threadIdx.x & 63;
  const int64_t p = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  if (p >= npieces) return;
  const int32_t r = piece_seg[p];
  const int32_t k = (int32_t)p - a.piece0[r];
  if (k == 0) return;
  const int32_t beg = a.fptr[r] + k * a.seg_len;
  const int32_t end = min(beg + a.seg_len, a.fptr[r + 1]);
  const int32_t slot = beg + lane;
  const bool ok = slot < end;
  const int32_t n = a.fnbr[ok ? slot : beg];
  float acc[8];
#pragma unroll
  for (int f = 0; f < 8; ++f) {
    float v[1] = {(ok && f < a.F) ? a.x[(int64_t)n * a.ldx + f] : 0.0f};
    if (ok && f < a.F) contrib<MODE, 1>(a, n, r, slot, f, v);
    acc[f] = v[0];
  }
#pragma unroll
  for (int f = 0; f < 8; ++f)
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) acc[f] += __shfl_xor(acc[f], off);
  if (lane == 0) {
#pragma unroll
    for (int f = 0; f < 8; ++f)
      if (f < a.F) a.part[p * a.F + f] = acc[f];
  }
}

// Combine: one wave per long segment, its pieces' partials added in piece order, then the
// mode's finish (mean divide, root addend, bias, ReLU) and the store.
template <int MODE, int VEC, int NCH>
__global__ __launch_bounds__(256) void agg_combine_kernel(AggArgs a, int64_t nlong, const int32_t* long_seg) {
  const int lane = threadIdx.x & 63;
  const int64_t l = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  if (l >= nlong) return;
  const int32_t r = long_seg[l];
  const int32_t p0 = a.piece0[r];
  const int32_t deg = a.fptr[r + 1] - a.fptr[r];
  const int32_t np = (deg + a.seg_len - 1) / a.seg_len;
  const int nchunk = a.F / VEC;
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c = lane + 64 * i;
    if (c >= nchunk) continue;
    float acc[VEC];
    vload<VEC>(a.part + (int64_t)p0 * a.F + c * VEC, acc);
    for (int32_t k = 1; k < np; ++k) {
      float t[VEC];
      vload<VEC>(a.part + (int64_t)(p0 + k) * a.F + c * VEC, t);
#pragma unroll
      for (int q = 0; q < VEC; ++q) acc[q] += t[q];
    }
    finish<MODE, VEC>(a, r, c * VEC, acc);
    vstore<VEC>(a.y + (int64_t)r * a.ldy + c * VEC, acc);
  }
}

bool aligned(const void* p, int bytes) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) % bytes) == 0; }

// Kernel-lab knob: the constant 0 in libgnnmp.so (no global mutable state, no lab kernels
// instantiated).  `make lab` compiles this file again with -DGNNMP_AGG_LAB into
// _lab/libgnnmp_agglab.so, whose gnnx_set_agg_variant selects the lab launch shapes
// (profiles/lab_agg.py, lab_order.py, tests/test_gpu_order.py).
#ifdef GNNMP_AGG_LAB
int g_agg_lab_variant = 0;
#else
constexpr int g_agg_lab_variant = 0;
#endif

template <int MODE, int VEC, int NCH>
void launch_split_passes(const AggArgs& a, const gnn_split* sp, hipStream_t st) {
  if (sp->num_pieces > sp->num_long)
    agg_piece_wide_kernel<MODE, VEC, NCH><<<(unsigned)ceil_div(sp->num_pieces * 64, 256), 256, 0, st>>>(
        a, sp->num_pieces, sp->piece_seg);
  agg_combine_kernel<MODE, VEC, NCH><<<(unsigned)ceil_div(sp->num_long * 64, 256), 256, 0, st>>>(
      a, sp->num_long, sp->long_seg);
}

template <int MODE, int VEC>
void launch_split_v(const AggArgs& a, const gnn_split* sp, hipStream_t st) {
  const int nch = (int)ceil_div(a.F / VEC, 64);
  // (r12: 16- / 32-lane groups per piece and per combined row, 4 / 2 per wave, measured 6 us slower
  // per F = 64 pass than one wave each — per-lane id loads and divergent piece lengths)
  if (nch <= 1) launch_split_passes<MODE, VEC, 1>(a, sp, st);
  else if (nch <= 2) launch_split_passes<MODE, VEC, 2>(a, sp, st);
  else launch_split_passes<MODE, VEC, 4>(a, sp, st);
}


template <int MODE>
gnn_status launch_mode(const AggArgs& a, int vec, hipStream_t st, const gnn_split* sp,
                       const gnn_split* pieces = nullptr, bool* pieces_done = nullptr);

template <int MODE>
gnn_status launch_mode_split(const AggArgs& a, int vec, hipStream_t st, const gnn_split* sp) {
  bool pieces_done = false;  // the lane-group main pass takes the pieces into its own launch
  gnn_status s = launch_mode<MODE>(a, vec, st, nullptr, sp, &pieces_done);  // main pass over the truncated segments
  if (s != GNN_OK || sp->num_long == 0) return s;
  if (pieces_done) {
    const int nch = (int)ceil_div(a.F / vec, 64);
    if (vec == 4 && nch <= 1) agg_combine_kernel<MODE, 4, 1><<<(unsigned)ceil_div(sp->num_long * 64, 256), 256, 0, st>>>(a, sp->num_long, sp->long_seg);
    else if (vec == 2 && nch <= 1) agg_combine_kernel<MODE, 2, 1><<<(unsigned)ceil_div(sp->num_long * 64, 256), 256, 0, st>>>(a, sp->num_long, sp->long_seg);
    else agg_combine_kernel<MODE, 1, 1><<<(unsigned)ceil_div(sp->num_long * 64, 256), 256, 0, st>>>(a, sp->num_long, sp->long_seg);
    return hip_check(hipGetLastError(), "gnn_aggregate_f32 (split combine)");
  }
  if (a.F <= 8) {
    if (sp->num_pieces > sp->num_long)
      agg_piece_narrow_kernel<MODE><<<(unsigned)ceil_div(sp->num_pieces * 64, 256), 256, 0, st>>>(
          a, sp->num_pieces, sp->piece_seg);
    agg_combine_kernel<MODE, 1, 1><<<(unsigned)ceil_div(sp->num_long * 64, 256), 256, 0, st>>>(
        a, sp->num_long, sp->long_seg);
  } else if (vec == 4) {
    launch_split_v<MODE, 4>(a, sp, st);
  } else if (vec == 2) {
    launch_split_v<MODE, 2>(a, sp, st);
  } else {
    launch_split_v<MODE, 1>(a, sp, st);
  }
  return hip_check(hipGetLastError(), "gnn_aggregate_f32 (split passes)");
}

template <int MODE>
gnn_status launch_mode(const AggArgs& a, int vec, hipStream_t st, const gnn_split* sp, const gnn_split* pieces,
                       bool* pieces_done) {
  if (a.nrows == 0 || a.F == 0) return GNN_OK;
  if (sp) return launch_mode_split<MODE>(a, vec, st, sp);
  if ((a.F <= 4 && (MODE == GNN_AGG_MEAN || MODE == GNN_AGG_MEAN_BWD || MODE == GNN_AGG_SUM)) ||
      (a.F <= 2 && MODE == GNN_AGG_GCN)) {  // (GCN: the 2-class logits and their transpose, r54)
    // slots staged per pass: 512 / 128 measured 15.3 / 17.2 us vs 16.1 at 256 (r10, warm)
    const unsigned nb = (unsigned)ceil_div(a.nrows, 256);
    // rows longer than 32 slots of a pass: the tail by the whole wave (r17 lab, SAGE preset F = 2:
    // fwd 14.4 -> 13.2 us, CSC bwd 15.2 -> 14.4 cold); lab 15: each lane walks its whole row
#ifdef GNNMP_AGG_LAB
    if (g_agg_lab_variant == 15) {
      if (a.F <= 2) agg_narrow_lds_kernel<MODE, 2, 256, false><<<nb, 256, 0, st>>>(a);
      else if constexpr (MODE != GNN_AGG_GCN) agg_narrow_lds_kernel<MODE, 4, 256, false><<<nb, 256, 0, st>>>(a);
    } else
#endif
    if (a.F <= 2) agg_narrow_lds_kernel<MODE, 2, 256, true><<<nb, 256, 0, st>>>(a);
    else if constexpr (MODE != GNN_AGG_GCN) agg_narrow_lds_kernel<MODE, 4, 256, true><<<nb, 256, 0, st>>>(a);
  } else if (a.F <= 8) {
    int64_t blocks = ceil_div(a.nrows * kGroup, 256);
    if (blocks > ((int64_t)1 << 20)) blocks = (int64_t)1 << 20;
    if (a.F <= 2) agg_group_kernel<MODE, 2><<<(unsigned)blocks, 256, 0, st>>>(a);
    else if (a.F <= 4) agg_group_kernel<MODE, 4><<<(unsigned)blocks, 256, 0, st>>>(a);
    else agg_group_kernel<MODE, 8><<<(unsigned)blocks, 256, 0, st>>>(a);
  } else {
    const int nchunk = a.F / vec;
    int lps = 64;
    if (nchunk <= 8) lps = 8;
    else if (nchunk <= 16) lps = 16;
    else if (nchunk <= 32) lps = 32;
    if (nchunk > 64 * 4) return fail(GNN_ERR_UNSUPPORTED, "gnn_aggregate_f32", "F too wide for the gather kernel");
    // rows per group: the group's lanes hold rpg + 1 row pointers, so rpg <= lps - 1.  16-lane
    // groups (F = 64): 2 rows — the 4 groups of a wave walk their rows in lockstep more often and
    // flush (divergently) fewer rows per pass: GCN preset F = 64, CSR fwd with bias / ReLU /
    // dropout 97.5 -> 89.2 us, CSC bwd 49.4 -> 41.3 us (profiles/lab_agg.py, r08; 4 rows: 91.5 /
    // 41.7, lps - 1 = 15 rows: 116.9 / 48.7).  Lab 5 / 6 / 8: 4 / 8 / lps - 1 rows.
    const int lv = g_agg_lab_variant;
    // degree-ordered split main pass (a.order): ONE row per group — a wave's groups hold rows of
    // the same length, so they walk in lockstep and nothing is gained by walking several rows
    // flat; more, shorter-lived groups hide more latency (r14 lab, F = 64: SAGE mean fwd 59.7 ->
    // 50.3 us, CSC mean bwd 80.0 -> 62.9, GCN fwd 73.5 -> 59.1; plan order at 2 rows: 71 / 98 / 84)
    const int rpg = lv == 5 ? 4 : lv == 6 ? 8 : lv == 8 ? lps - 1 : (lv == 9 || lv == 11) ? 1
                  : a.order ? 1 : (lps == 8 ? 7 : lps == 16 ? 2 : 8);
    const int64_t groups = ceil_div(a.nrows, rpg);
    const unsigned blocks = (unsigned)ceil_div(groups * lps, 256);
    const bool pf = lv == 10 || lv == 11;  // lab: neighbour-id prefetch (r14: 5-10 us slower)
    // split pieces (one wave each) folded into the main pass's launch: 16-lane groups only (r17:
    // F = 64 passes 10-12 us faster; at F = 128 (32-lane groups) the scaled config's CSC pass
    // measured 1463 -> 1679 us, the pieces' registers lowering the main pass's occupancy)
    const bool fold = pieces && pieces->num_pieces > pieces->num_long && !pf && lps == 16 && lv != 16;
    const unsigned pblocks = fold ? (unsigned)ceil_div(pieces->num_pieces * 64, 256) : 0u;
    if (fold && pieces_done) *pieces_done = true;
#ifdef GNNMP_AGG_LAB
#define GNN_FLAT_PF(V, L, NC) if (pf) agg_flat_kernel<MODE, V, L, NC, true><<<blocks, 256, 0, st>>>(a, rpg); else
#else
#define GNN_FLAT_PF(V, L, NC)
#endif
#define GNN_FLAT(V, L, NC)                                                                                 \
  do {                                                                                                     \
    GNN_FLAT_PF(V, L, NC)                                                                                  \
    if (fold)                                                                                              \
      agg_flat_pieces_kernel<MODE, V, L, NC><<<blocks + pblocks, 256, 0, st>>>(a, rpg, pieces->num_pieces,   \
                                                                           pieces->piece_seg, pblocks);    \
    else agg_flat_kernel<MODE, V, L, NC><<<blocks, 256, 0, st>>>(a, rpg);                                    \
  } while (0)
#define GNN_FLAT_V(V)                      \
  do {                                     \
    if (lps == 64) GNN_FLAT(V, 64, 4);     \
    else if (lps == 32) GNN_FLAT(V, 32, 1); \
    else if (lps == 16) GNN_FLAT(V, 16, 1); \
    else GNN_FLAT(V, 8, 1);                \
  } while (0)
    if (lps == 64 && nchunk <= 128) {  // wave-uniform fast path (scalar row/neighbour handling)
      // 16 rows per wave.  r08 lab (profiles/lab_agg.py, SAGE preset F = 166 CSR, 89.4 us = 63 %
      // of HBM): 8 rows 89.2, 4 rows 95.7, 32 rows 99.1; U = 4 rows in flight 91.9; a 168-float
      // padded pitch (dwordx4, one load per row) 89.0 — the gather is not instruction-bound.
      // XCD-grouped block order (each XCD sweeping one contiguous eighth of the rows) measured
      // slower with cold caches (r10: 130.4 -> 138.5 us).  Lab 1 / 2 / 3: 8 / 4 / 32 rows.
      const int rpw = (lv == 1 || lv == 14) ? 8 : (lv == 2 || lv == 13) ? 4 : lv == 3 ? 32 : 16;
      const unsigned wblocks = (unsigned)ceil_div(ceil_div(a.nrows, rpw) * 64, 256);
      // (r13 lab: U = 16 neighbour rows in flight instead of 8, 98.5 -> 308.7 us warm — register
      // pressure; not kept)
      if (vec == 4) agg_wave_kernel<MODE, 4, 2, false, 8><<<wblocks, 256, 0, st>>>(a, rpw);
      else if (vec == 2) agg_wave_kernel<MODE, 2, 2, false, 8><<<wblocks, 256, 0, st>>>(a, rpw);
      else agg_wave_kernel<MODE, 1, 2, false, 8><<<wblocks, 256, 0, st>>>(a, rpw);
    } else if (vec == 4) GNN_FLAT_V(4);
    else if (vec == 2) GNN_FLAT_V(2);
    else GNN_FLAT_V(1);
#undef GNN_FLAT_V
#undef GNN_FLAT
#undef GNN_FLAT_PF
  }
  return hip_check(hipGetLastError(), "gnn_aggregate_f32");
}

// ------------------------------------------------------------------ colsum
// Stage 1: block b sums rows [b*rpb, (b+1)*rpb); threads form (row lanes x columns) so that
// narrow F still uses the whole block; each thread keeps 4 independent accumulators (4 row
// loads in flight), combined in a fixed order, then row-lane partials combine in LDS.
__global__ __launch_bounds__(256) void colsum_partial_kernel(int64_t rows, int32_t F, const float* __restrict__ x,
                                                             int64_t ldx, int64_t rows_per_blk,
                                                             float* __restrict__ part) {
  __shared__ float red[256];
  const int cols = F < 256 ? F : 256;
  const int lanes = 256 / cols;  // row lanes per column
  const int c_local = threadIdx.x % cols;
  const int rl = threadIdx.x / cols;
  const int64_t r0 = blockIdx.x * rows_per_blk;
  const int64_t r1 = r0 + rows_per_blk < rows ? r0 + rows_per_blk : rows;
  for (int cb = 0; cb < F; cb += cols) {
    const int c = cb + c_local;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    if (rl < lanes && c < F) {
      int64_t r = r0 + rl;
      for (; r + 3 * lanes < r1; r += 4 * lanes) {
        a0 += x[r * ldx + c];
        a1 += x[(r + lanes) * ldx + c];
        a2 += x[(r + 2 * lanes) * ldx + c];
        a3 += x[(r + 3 * lanes) * ldx + c];
      }
      for (; r < r1; r += lanes) a0 += x[r * ldx + c];
    }
    red[threadIdx.x] = (a0 + a1) + (a2 + a3);
    __syncthreads();
    if (threadIdx.x < cols && cb + (int)threadIdx.x < F) {
      float s = 0.0f;
      for (int l = 0; l < lanes; ++l) s += red[l * cols + threadIdx.x];
      part[(int64_t)blockIdx.x * F + cb + threadIdx.x] = s;
    }
    __syncthreads();
  }
}

// Stage 2: one block per column; 256 threads stride the partials (4 loads in flight each),
// then a fixed-shape LDS tree.  Deterministic.
__global__ __launch_bounds__(256) void colsum_final_kernel(int32_t F, int32_t nblk, const float* __restrict__ part,
                                                           float* __restrict__ out) {
  __shared__ float red[256];
  const int c = blockIdx.x;
  const int t = threadIdx.x;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int b = t;
  for (; b + 768 < nblk; b += 1024) {
    a0 += part[(int64_t)b * F + c];
    a1 += part[(int64_t)(b + 256) * F + c];
    a2 += part[(int64_t)(b + 512) * F + c];
    a3 += part[(int64_t)(b + 768) * F + c];
  }
  for (; b < nblk; b += 256) a0 += part[(int64_t)b * F + c];
  red[t] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (t < s) red[t] += red[t + s];
    __syncthreads();
  }
  if (t == 0) out[c] = red[0];
}

constexpr int64_t kColsumBlocks = 1024;

}  // namespace
}  // namespace gnnmp

using namespace gnnmp;

#ifdef GNNMP_AGG_LAB
// Lab build only (not in libgnnmp.so): selects lab launch shapes of the gathers.
extern "C" void gnnx_set_agg_variant(int v) { g_agg_lab_variant = v; }
#endif

extern "C" gnn_status gnn_aggregate_f32(const gnn_graph* g, const gnn_agg_params* p, const float* x,
                                        int64_t ldx, int64_t F, float* y, int64_t ldy,
                                        gnn_stream_t stream) {
  if (!g || !p) return fail(GNN_ERR_INVALID_ARG, __func__, "null graph or params");
  if (F < 0 || F > INT32_MAX || ldx < F || ldy < F)
    return fail(GNN_ERR_INVALID_ARG, __func__, "bad F / leading dimensions");
  if (g->num_nodes > 0 && F > 0 && (!x || !y)) return fail(GNN_ERR_INVALID_ARG, __func__, "null x/y");
  if (p->addend && p->ld_add < F) return fail(GNN_ERR_INVALID_ARG, __func__, "bad ld_add");
  if (p->addend2 && p->ld_add2 < F) return fail(GNN_ERR_INVALID_ARG, __func__, "bad ld_add2");
  AggArgs a{};
  a.ptr = p->transpose ? g->colptr : g->rowptr;
  a.nbr = p->transpose ? g->row : g->col;
  a.wslot = (p->mode == GNN_AGG_EDGE_W && p->transpose) ? g->csc2csr : nullptr;
  a.nodew = p->nodew;
  a.ew = p->ew;
  a.heads = p->heads > 0 ? p->heads : 1;
  a.x = x; a.ldx = ldx; a.y = y; a.ldy = ldy;
  a.add = p->addend; a.ld_add = p->ld_add;
  a.add2 = p->addend2; a.ld_add2 = p->ld_add2;
  a.bias = p->bias; a.relu = p->relu;
  if (p->dropout_p < 0.f || p->dropout_p >= 1.f) return fail(GNN_ERR_INVALID_ARG, __func__, "dropout p in [0,1)");
  if (p->dropout_p > 0.f && (int64_t)g->num_nodes * (int64_t)F >= ((int64_t)1 << 32))
    return fail(GNN_ERR_UNSUPPORTED, __func__, "dropout element index (rows x width) must be < 2^32");
  a.dropout = p->dropout_p > 0.f;
  a.keep_thresh = (uint32_t)((1.0 - (double)p->dropout_p) * 16777216.0);
  a.drop_scale = a.dropout ? (float)(1.0 / (1.0 - (double)p->dropout_p)) : 1.0f;
  a.seed = p->seed;
  a.seed_ptr = p->seed_ptr;
  a.nrows = g->num_nodes;
  a.F = (int32_t)F;
  if (!a.ptr || (g->num_slots > 0 && !a.nbr)) return fail(GNN_ERR_INVALID_ARG, __func__, "plan arrays null");
  if ((p->mode == GNN_AGG_MEAN || p->mode == GNN_AGG_MEAN_BWD || p->mode == GNN_AGG_GCN) && !p->nodew)
    return fail(GNN_ERR_INVALID_ARG, __func__, "mode needs nodew");
  if (p->mode == GNN_AGG_EDGE_W) {
    if (!p->ew) return fail(GNN_ERR_INVALID_ARG, __func__, "EDGE_W needs ew");
    if (F % a.heads) return fail(GNN_ERR_INVALID_ARG, __func__, "F not divisible by heads");
    if (p->transpose && !g->csc2csr) return fail(GNN_ERR_INVALID_ARG, __func__, "EDGE_W transpose needs csc2csr");
  }
  a.chan = (int32_t)(F / a.heads > 0 ? F / a.heads : 1);
  auto ok_vec = [&](int v) {
    if (F % v || ldx % v || ldy % v) return false;
    if (p->addend && p->ld_add % v) return false;
    if (p->addend2 && p->ld_add2 % v) return false;
    if (p->mode == GNN_AGG_EDGE_W && a.chan % v) return false;
    int b = 4 * v;
    return aligned(x, b) && aligned(y, b) && aligned(p->addend, b) && aligned(p->addend2, b);
  };
  // Long-segment split (not for EDGE_W: its weights are indexed by the untruncated slot).
  const gnn_split* sp = p->transpose ? g->csc_split : g->csr_split;
  if (sp && (p->mode == GNN_AGG_EDGE_W || !p->part || sp->seg_len < 1 || sp->seg_len > 64 ||
             p->part_bytes < (size_t)sp->num_pieces * (size_t)F * sizeof(float) ||
             (sp->num_long > 0 && (!sp->ptr || !sp->nbr || !sp->piece0 || !sp->piece_seg || !sp->long_seg))))
    sp = nullptr;  // unsplit fallback is always correct
  if (sp) {
    a.fptr = a.ptr;
    a.fnbr = a.nbr;
    a.ptr = sp->ptr;
    a.nbr = sp->nbr;
    a.piece0 = sp->piece0;
    a.order = sp->order;
    a.part = p->part;
    a.seg_len = sp->seg_len;
  }
  int vec = ok_vec(4) ? 4 : (ok_vec(2) ? 2 : 1);
  while (sp && vec > 1 && !aligned(p->part, 4 * vec)) vec >>= 1;
  // The split pays only for the lane-group gather (8..32 lanes per row, one row at a time per
  // group): r01 measurements — F=64 GCN fwd 72 -> 37 µs; the wave-wide gather (F/vec > 32) and
  // the narrow LDS/group kernels lose to the two extra launches.
  // (lab 12 / 13 / 14: the split, degree-ordered, for the wave-wide gather too, 16 / 4 / 8 rows per wave)
  const bool lab_wsplit = g_agg_lab_variant >= 12 && g_agg_lab_variant <= 14;
  if (sp && (F <= 8 || (F / vec > 32 && !lab_wsplit) || g_agg_lab_variant == 7)) sp = nullptr;  // lab 7: no split
  if (!sp) {
    a.ptr = p->transpose ? g->colptr : g->rowptr;
    a.nbr = p->transpose ? g->row : g->col;
    a.piece0 = nullptr;
    a.order = nullptr;
    a.part = nullptr;
  }
  hipStream_t st = (hipStream_t)stream;
  switch (p->mode) {
    case GNN_AGG_SUM: return launch_mode<GNN_AGG_SUM>(a, vec, st, sp);
    case GNN_AGG_MEAN: return launch_mode<GNN_AGG_MEAN>(a, vec, st, sp);
    case GNN_AGG_MEAN_BWD: return launch_mode<GNN_AGG_MEAN_BWD>(a, vec, st, sp);
    case GNN_AGG_GCN: return launch_mode<GNN_AGG_GCN>(a, vec, st, sp);
    case GNN_AGG_EDGE_W: return launch_mode<GNN_AGG_EDGE_W>(a, vec, st, nullptr);
  }
  return fail(GNN_ERR_INVALID_ARG, __func__, "unknown mode");
}

// bf16-storage aggregation: x and y bf16 ([rows, F], ld in elements), f32 accumulation in plan
// order, y rounded once (RNE).  Modes SUM / MEAN / MEAN_BWD / GCN; addend (f32), bias, ReLU as
// in gnn_aggregate_f32; no long-segment split.  F <= 512.
namespace gnnmp {
namespace {
// lane groups of the bf16 gather (agg_wave_group_bf16_kernel): 2 = two slots per load instruction
// (VEC 4, F / 4 <= 32: configs[4]'s F = 128 mean 609 -> 496 us), 1 = one (agg_wave_kernel, 32 of 64
// lanes at F = 128), 4 = four (VEC 8, F / 8 <= 16: measured slower, 786 us at occupancy 4 —
// profiles/r99_bf_groups.txt; two groups over 16-byte pieces for the 168-wide layer-0 rows also
// measured slower, +130-180 us per step); GNNMP_BF_GROUPS overrides (A/B)
int bf16_groups() {
  static const int v = [] {
    const char* e = std::getenv("GNNMP_BF_GROUPS");
    return e ? std::atoi(e) : 2;
  }();
  return v;
}

template <int MODE>
gnn_status launch_bf16(const AggArgs& a, int vec, bool vec8, hipStream_t st) {
  if (a.nrows == 0 || a.F == 0) return GNN_OK;
  const int rpw = 16;
  const unsigned wblocks = (unsigned)ceil_div(ceil_div(a.nrows, rpw) * 64, 256);
  const int nchunk = a.F / vec;
  if constexpr (MODE != GNN_AGG_GCN) {
    const int grp = bf16_groups();
    if (grp == 4 && vec8 && a.F / 8 <= 16) {
      agg_wave_group_bf16_kernel<MODE, 8, 4, 4><<<wblocks, 256, 0, st>>>(a, rpw);
      return hip_check(hipGetLastError(), "gnn_aggregate_bf16");
    }
    if (grp >= 2 && vec == 4 && nchunk <= 32) {
      agg_wave_group_bf16_kernel<MODE, 4, 2><<<wblocks, 256, 0, st>>>(a, rpw);
      return hip_check(hipGetLastError(), "gnn_aggregate_bf16");
    }
  }
  if (nchunk <= 64) {
    if (vec == 4) agg_wave_kernel<MODE, 4, 1, true><<<wblocks, 256, 0, st>>>(a, rpw);
    else if (vec == 2) agg_wave_kernel<MODE, 2, 1, true><<<wblocks, 256, 0, st>>>(a, rpw);
    else agg_wave_kernel<MODE, 1, 1, true><<<wblocks, 256, 0, st>>>(a, rpw);
  } else {
    if (vec == 4) agg_wave_kernel<MODE, 4, 2, true><<<wblocks, 256, 0, st>>>(a, rpw);
    else if (vec == 2) agg_wave_kernel<MODE, 2, 2, true><<<wblocks, 256, 0, st>>>(a, rpw);
    else agg_wave_kernel<MODE, 1, 2, true><<<wblocks, 256, 0, st>>>(a, rpw);
  }
  return hip_check(hipGetLastError(), "gnn_aggregate_bf16");
}

}  // namespace
}  // namespace gnnmp

extern "C" gnn_status gnn_aggregate_bf16(const gnn_graph* g, const gnn_agg_params* p, const void* x, int64_t ldx,
                                         int64_t F, void* y, int64_t ldy, gnn_stream_t stream) {
  if (!g || !p) return fail(GNN_ERR_INVALID_ARG, __func__, "null graph or params");
  if (F < 0 || ldx < F || ldy < F) return fail(GNN_ERR_INVALID_ARG, __func__, "bad F / leading dimensions");
  if (p->mode == GNN_AGG_EDGE_W) return fail(GNN_ERR_UNSUPPORTED, __func__, "EDGE_W has no bf16 form");
  if ((p->mode == GNN_AGG_MEAN || p->mode == GNN_AGG_MEAN_BWD || p->mode == GNN_AGG_GCN) && !p->nodew)
    return fail(GNN_ERR_INVALID_ARG, __func__, "mode needs nodew");
  if (g->num_nodes > 0 && F > 0 && (!x || !y)) return fail(GNN_ERR_INVALID_ARG, __func__, "null x/y");
  if (p->addend && p->ld_add < F) return fail(GNN_ERR_INVALID_ARG, __func__, "bad ld_add");
  if (p->addend2) return fail(GNN_ERR_UNSUPPORTED, __func__, "addend2 is f32-only");
  AggArgs a{};
  a.ptr = p->transpose ? g->colptr : g->rowptr;
  a.nbr = p->transpose ? g->row : g->col;
  if (!a.ptr || (g->num_slots > 0 && !a.nbr)) return fail(GNN_ERR_INVALID_ARG, __func__, "plan arrays null");
  a.nodew = p->nodew;
  a.heads = 1;
  a.chan = (int32_t)(F > 0 ? F : 1);
  a.x = static_cast<const float*>(x); a.ldx = ldx;
  a.y = static_cast<float*>(y); a.ldy = ldy;
  a.add = p->addend; a.ld_add = p->ld_add;
  a.bias = p->bias; a.relu = p->relu;
  if (p->dropout_p < 0.f || p->dropout_p >= 1.f) return fail(GNN_ERR_INVALID_ARG, __func__, "dropout p in [0,1)");
  if (p->dropout_p > 0.f && (int64_t)g->num_nodes * (int64_t)F >= ((int64_t)1 << 32))
    return fail(GNN_ERR_UNSUPPORTED, __func__, "dropout element index (rows x width) must be < 2^32");
  a.dropout = p->dropout_p > 0.f;
  a.keep_thresh = (uint32_t)((1.0 - (double)p->dropout_p) * 16777216.0);
  a.drop_scale = a.dropout ? (float)(1.0 / (1.0 - (double)p->dropout_p)) : 1.0f;
  a.seed = p->seed;
  a.seed_ptr = p->seed_ptr;
  a.nrows = g->num_nodes;
  a.F = (int32_t)F;
  auto ok_vec = [&](int v) {
    if (F % v || ldx % v || ldy % v || (p->addend && p->ld_add % v)) return false;
    return aligned(x, 2 * v) && aligned(y, 2 * v) && aligned(p->addend, 4 * v);
  };
  const int vec = ok_vec(4) ? 4 : (ok_vec(2) ? 2 : 1);
  const bool vec8 = ok_vec(8);
  if (F / vec > 128) return fail(GNN_ERR_UNSUPPORTED, __func__, "F too wide for the bf16 gather");
  hipStream_t st = (hipStream_t)stream;
  switch (p->mode) {
    case GNN_AGG_SUM: return launch_bf16<GNN_AGG_SUM>(a, vec, vec8, st);
    case GNN_AGG_MEAN: return launch_bf16<GNN_AGG_MEAN>(a, vec, vec8, st);
    case GNN_AGG_MEAN_BWD: return launch_bf16<GNN_AGG_MEAN_BWD>(a, vec, vec8, st);
    case GNN_AGG_GCN: return launch_bf16<GNN_AGG_GCN>(a, vec, vec8, st);
    default: return fail(GNN_ERR_INVALID_ARG, __func__, "unknown mode");
  }
}

extern "C" gnn_status gnn_sage_mean_fwd_f32(const gnn_graph* g, const float* deg, const float* x,
                                            int64_t ldx, int64_t F, float* out, int64_t ldo,
                                            gnn_stream_t stream) {
  gnn_agg_params p{};
  p.mode = GNN_AGG_MEAN;
  p.transpose = 0;
  p.nodew = deg;
  return gnn_aggregate_f32(g, &p, x, ldx, F, out, ldo, stream);
}

// K1 with a split-image store: y = mean_{j->i} x[j] (MEAN over the CSR rows, PyG's order and
// rounding) written as 3 bf16 planes (hi = RNE(y), mid = RNE(y - hi), lo = RNE(y - hi - mid)) or,
// PLN = 2, as 2 f16 planes (hi = RNE_f16(y), lo = RNE_f16((y - hi)·2^11)) at img + p·plane_stride,
// row pitch ld, columns [F, width) zero.  Wide rows only (the wave gather).
template <int PLN>
static gnn_status sage_mean_fwd_image(const gnn_graph* g, const float* deg, const float* x, int64_t ldx, int64_t F,
                                      void* img, int64_t ld, int64_t plane_stride, int64_t width, gnn_stream_t stream,
                                      const char* fn, uint32_t* keep_mask = nullptr, int64_t mask_cols = 0,
                                      float dropout_p = 0.f, uint64_t seed = 0, const uint64_t* seed_ptr = nullptr,
                                      const gnn_gemm_nt_params* prep_b = nullptr, int32_t scale_exp = 0,
                                      const gnn_split* hub = nullptr) {
  if (!g || !deg) return fail(GNN_ERR_INVALID_ARG, fn, "null graph or deg");
  if (scale_exp < -100 || scale_exp > 100) return fail(GNN_ERR_INVALID_ARG, fn, "scale_exp outside [-100, 100]");
  if (F < 2 || ldx < F || width < F || width > ld || plane_stride < g->num_nodes * ld)
    return fail(GNN_ERR_INVALID_ARG, fn, "bad F / width / leading dimensions");
  if (g->num_nodes > 0 && (!x || !img)) return fail(GNN_ERR_INVALID_ARG, fn, "null x / image");
  if (!g->rowptr || (g->num_slots > 0 && !g->col)) return fail(GNN_ERR_INVALID_ARG, fn, "plan arrays null");
  AggArgs a{};
  a.ptr = g->rowptr;
  a.nbr = g->col;
  a.nodew = deg;
  a.heads = 1;
  a.chan = (int32_t)F;
  a.x = x; a.ldx = ldx;
  a.yp = static_cast<uint16_t*>(img); a.ldy = ld; a.yps = plane_stride; a.ywidth = (int32_t)width;
  a.yscale = ldexpf(1.0f, scale_exp);
  a.nrows = g->num_nodes;
  a.F = (int32_t)F;
  if (keep_mask) {
    if (mask_cols < 1 || mask_cols > 128 || !(dropout_p > 0.f && dropout_p < 1.f) ||
        (reinterpret_cast<uintptr_t>(keep_mask) & 15) || g->num_nodes * mask_cols >= ((int64_t)1 << 32))
      return fail(GNN_ERR_INVALID_ARG, fn, "keep mask: 1 <= mask_cols <= 128, 0 < p < 1, 16-byte aligned, rows x cols < 2^32");
    a.kmask = keep_mask; a.kcols = (int32_t)mask_cols;
    a.dropout = 1;
    a.keep_thresh = (uint32_t)((1.0 - (double)dropout_p) * 16777216.0);
    a.seed = seed;
    a.seed_ptr = reinterpret_cast<const int64_t*>(seed_ptr);
  }
  if (prep_b) {  // the half-pair NT that reads this image: its B prep joins this launch
    if (PLN != 2 || prep_b->a_planes != img || prep_b->planes_exp != scale_exp)
      return fail(GNN_ERR_INVALID_ARG, fn, "prep_b: the NT must read this half-pair image (same planes_exp)");
    const gnn_status s = nt_h2_prep_from_params(prep_b, &a.hp, fn);
    if (s != GNN_OK) return s;
    a.hp.gblocks = BN / 4;  // one wave per output column (ws_prep_h2_cols<256>)
  }
  auto al = [](const void* q, int b) { return (reinterpret_cast<uintptr_t>(q) % b) == 0; };
  const bool v4 = F % 4 == 0 && ldx % 4 == 0 && width % 4 == 0 && ld % 4 == 0 && plane_stride % 4 == 0 &&
                  al(x, 16) && al(img, 8);
  const bool v2 = F % 2 == 0 && ldx % 2 == 0 && width % 2 == 0 && ld % 2 == 0 && plane_stride % 2 == 0 &&
                  al(x, 8) && al(img, 4);
  const int vec = v4 ? 4 : 2;
  if (!v2 || F / vec <= 32 || ceil_div(width, vec) > 128)
    return fail(GNN_ERR_UNSUPPORTED, fn, "needs even F, 32 < F / vec, width / vec <= 128 and aligned rows");
  if (hub && hub->num_long > 0) {  // the hub form: hub rows on blocks of their own
    if (PLN != 2 || hub->order || hub->piece0 || !hub->ptr || !hub->long_seg || hub->seg_len < 1 ||
        hub->num_long > g->num_nodes || (!hub->nbr && g->num_slots > 0))
      return fail(GNN_ERR_INVALID_ARG, fn, "hub: a natural-order split (order, piece0 NULL) with ptr, nbr, long_seg, seg_len >= 1");
    a.fptr = g->rowptr; a.fnbr = g->col;
    a.ptr = hub->ptr; a.nbr = hub->nbr;
    a.hubs = hub->long_seg; a.nhub = (int32_t)hub->num_long; a.hub_deg = (float)hub->seg_len;
  }
  if (hub && hub->piece_seg) {  // balanced main-pass waves (validated by the plan that built them)
    if (PLN != 2 || hub->order || hub->piece0 || hub->num_pieces < 1 || hub->num_pieces > g->num_nodes)
      return fail(GNN_ERR_INVALID_ARG, fn, "hub wave starts: 1 <= num_pieces <= num_nodes, natural order");
    a.wstart = hub->piece_seg;
  }
  if (a.nrows == 0) return GNN_OK;
  const int rpw = a.wstart ? (int)hub->num_pieces : 16;  // (balanced: the kernel's rpg is the wave count)
  const int64_t nwaves = a.wstart ? hub->num_pieces : ceil_div(a.nrows, 16);
  const unsigned wblocks = (unsigned)ceil_div(nwaves * 64, 256) + (unsigned)a.hp.gblocks + (unsigned)a.nhub;
  hipStream_t st = (hipStream_t)stream;
  if (vec == 4 && ceil_div(width, 4) <= 64)  // one pass per row (e.g. a 168-wide padded x: 42 lanes)
    agg_wave_kernel<GNN_AGG_MEAN, 4, 1, false, 8, PLN><<<wblocks, 256, 0, st>>>(a, rpw);
  else if (vec == 4) agg_wave_kernel<GNN_AGG_MEAN, 4, 2, false, 8, PLN><<<wblocks, 256, 0, st>>>(a, rpw);
  else agg_wave_kernel<GNN_AGG_MEAN, 2, 2, false, 8, PLN><<<wblocks, 256, 0, st>>>(a, rpw);
  return hip_check(hipGetLastError(), fn);
}

extern "C" gnn_status gnn_sage_mean_fwd_planes(const gnn_graph* g, const float* deg, const float* x, int64_t ldx,
                                               int64_t F, void* img, int64_t ld, int64_t plane_stride, int64_t width,
                                               gnn_stream_t stream) {
  return sage_mean_fwd_image<3>(g, deg, x, ldx, F, img, ld, plane_stride, width, stream, __func__);
}

extern "C" gnn_status gnn_sage_mean_fwd_h2(const gnn_graph* g, const float* deg, const float* x, int64_t ldx,
                                           int64_t F, void* img, int64_t ld, int64_t plane_stride, int64_t width,
                                           int32_t scale_exp, uint32_t* keep_mask, int64_t mask_cols, float dropout_p,
                                           uint64_t seed, const uint64_t* seed_ptr, const gnn_gemm_nt_params* prep_b,
                                           const gnn_split* hub, gnn_stream_t stream) {
  return sage_mean_fwd_image<2>(g, deg, x, ldx, F, img, ld, plane_stride, width, stream, __func__, keep_mask,
                                mask_cols, dropout_p, seed, seed_ptr, prep_b, scale_exp, hub);
}

extern "C" gnn_status gnn_masked_ce_finish(const float* partial, int32_t nblk, float inv_denom, float* loss,
                                           gnn_stream_t stream);

extern "C" gnn_status gnn_sage_out_mean_ce_f32(const gnn_graph* g, const float* deg, const float* z, int64_t ldz,
                                               int32_t C, const float* bias, float* logits, int64_t ldo,
                                               const int64_t* y, const uint8_t* mask, const float* class_w,
                                               float inv_denom, float* dlogits, int64_t ld_d, float* u, int64_t ldu,
                                               float* colsum, float* loss, void* workspace, size_t workspace_bytes,
                                               gnn_stream_t stream) {
  const char* fn = __func__;
  if (!g || !deg) return fail(GNN_ERR_INVALID_ARG, fn, "null graph or deg");
  if (C < 1 || C > 4 || ldz < 2 * C || ldo < C || ld_d < C) return fail(GNN_ERR_INVALID_ARG, fn, "needs 1 <= C <= 4, ldz >= 2C");
  const int64_t N = g->num_nodes;
  if (N > 0 && (!z || !logits || !y || !mask || !class_w || !dlogits)) return fail(GNN_ERR_INVALID_ARG, fn, "null operand");
  if (!g->rowptr || (g->num_slots > 0 && !g->col)) return fail(GNN_ERR_INVALID_ARG, fn, "plan arrays null");
  const int nblk = (int)std::max<int64_t>(1, ceil_div(N, 256));
  if (!workspace || workspace_bytes < (size_t)nblk * sizeof(float)) return fail(GNN_ERR_WORKSPACE, fn, "workspace too small");
  hipStream_t st = (hipStream_t)stream;
  float* partial = static_cast<float*>(workspace);
  if (N == 0) {
    if (!loss) return hip_check(hipMemsetAsync(partial, 0, sizeof(float), st), fn);
    return hip_check(hipMemsetAsync(loss, 0, sizeof(float), st), fn);
  }
  AggArgs a{};
  a.ptr = g->rowptr; a.nbr = g->col; a.nodew = deg; a.heads = 1; a.chan = C;
  a.x = z; a.ldx = ldz; a.y = logits; a.ldy = ldo;
  a.add = z + C; a.ld_add = ldz; a.bias = bias;
  a.nrows = N; a.F = C;
  a.ce_y = y; a.ce_mask = mask; a.ce_w = class_w; a.ce_inv = inv_denom; a.ce_dl = dlogits; a.ce_ldd = ld_d;
  a.ce_part = partial;
  if (u && ldu < C) return fail(GNN_ERR_INVALID_ARG, fn, "ldu < C");
  a.ce_u = u; a.ce_ldu = ldu;
  a.ce_cs = colsum;
  if (C <= 2) agg_narrow_lds_kernel<GNN_AGG_MEAN, 2, 256, true, true><<<(unsigned)nblk, 256, 0, st>>>(a);
  else agg_narrow_lds_kernel<GNN_AGG_MEAN, 4, 256, true, true><<<(unsigned)nblk, 256, 0, st>>>(a);
  const gnn_status s = hip_check(hipGetLastError(), fn);
  if (s != GNN_OK || !loss) return s;  // loss NULL: the partials stay in the workspace (ClipAdam / finish)
  return gnn_masked_ce_finish(partial, nblk, inv_denom, loss, stream);
}

extern "C" gnn_status gnn_gcn_out_ce_f32(const gnn_graph* g, const float* dinv, const float* t, int64_t ldt,
                                         int32_t C, const float* bias, float* logits, int64_t ldo,
                                         const int64_t* y, const uint8_t* mask, const float* class_w,
                                         float inv_denom, float* dlogits, int64_t ld_d, float* colsum, float* loss,
                                         void* workspace, size_t workspace_bytes, gnn_stream_t stream) {
  const char* fn = __func__;
  if (!g || !dinv) return fail(GNN_ERR_INVALID_ARG, fn, "null graph or dinv");
  if (C < 1 || C > 2 || ldt < C || ldo < C || ld_d < C) return fail(GNN_ERR_INVALID_ARG, fn, "needs 1 <= C <= 2");
  const int64_t N = g->num_nodes;
  if (N < 1 || !t || !logits || !y || !mask || !class_w || !dlogits) return fail(GNN_ERR_INVALID_ARG, fn, "null operand / N < 1");
  if (!g->rowptr || (g->num_slots > 0 && !g->col)) return fail(GNN_ERR_INVALID_ARG, fn, "plan arrays null");
  const int nblk = (int)ceil_div(N, 256);
  if (!workspace || workspace_bytes < (size_t)nblk * sizeof(float)) return fail(GNN_ERR_WORKSPACE, fn, "workspace too small");
  hipStream_t st = (hipStream_t)stream;
  float* partial = static_cast<float*>(workspace);
  AggArgs a{};
  a.ptr = g->rowptr; a.nbr = g->col; a.nodew = dinv; a.heads = 1; a.chan = C;
  a.x = t; a.ldx = ldt; a.y = logits; a.ldy = ldo; a.bias = bias;
  a.nrows = N; a.F = C;
  a.ce_y = y; a.ce_mask = mask; a.ce_w = class_w; a.ce_inv = inv_denom; a.ce_dl = dlogits; a.ce_ldd = ld_d;
  a.ce_part = partial; a.ce_cs = colsum;
  agg_narrow_lds_kernel<GNN_AGG_GCN, 2, 256, true, true><<<(unsigned)nblk, 256, 0, st>>>(a);
  const gnn_status s = hip_check(hipGetLastError(), fn);
  if (s != GNN_OK || !loss) return s;
  return gnn_masked_ce_finish(partial, nblk, inv_denom, loss, stream);
}

extern "C" gnn_status gnn_sage_mean_bwd_f32(const gnn_graph* g, const float* deg, const float* dout,
                                            int64_t ld_dout, int64_t F, float* dx, int64_t ld_dx,
                                            gnn_stream_t stream) {
  gnn_agg_params p{};
  p.mode = GNN_AGG_MEAN_BWD;
  p.transpose = 1;
  p.nodew = deg;
  return gnn_aggregate_f32(g, &p, dout, ld_dout, F, dx, ld_dx, stream);
}

extern "C" gnn_status gnn_colsum_workspace_size(int64_t rows, int64_t F, size_t* bytes) {
  if (!bytes || rows < 0 || F < 0) return fail(GNN_ERR_INVALID_ARG, __func__, "bad args");
  *bytes = (size_t)kColsumBlocks * (size_t)(F > 0 ? F : 1) * sizeof(float);
  return GNN_OK;
}

extern "C" gnn_status gnn_colsum_finish_f32(const float* part, int32_t nblk, int64_t F, float* out,
                                             gnn_stream_t stream) {
  if (nblk < 1 || F < 1 || F > INT32_MAX || !part || !out) return fail(GNN_ERR_INVALID_ARG, __func__, "bad args");
  colsum_final_kernel<<<(unsigned)F, 256, 0, (hipStream_t)stream>>>((int32_t)F, nblk, part, out);
  return hip_check(hipGetLastError(), __func__);
}

extern "C" gnn_status gnn_colsum_f32(int64_t rows, int64_t F, const float* x, int64_t ldx, float* out,
                                     void* workspace, size_t workspace_bytes, gnn_stream_t stream) {
  if (rows < 0 || F < 0 || F > INT32_MAX || (F > 0 && !out) || ldx < F)
    return fail(GNN_ERR_INVALID_ARG, __func__, "bad args");
  if (F == 0) return GNN_OK;
  hipStream_t st = (hipStream_t)stream;
  if (rows == 0) return hip_check(hipMemsetAsync(out, 0, F * sizeof(float), st), __func__);
  int64_t nblk = rows < kColsumBlocks ? rows : kColsumBlocks;
  if (workspace_bytes < (size_t)nblk * F * sizeof(float) || !workspace)
    return fail(GNN_ERR_WORKSPACE, __func__, "workspace too small");
  int64_t rpb = ceil_div(rows, nblk);
  nblk = ceil_div(rows, rpb);
  float* part = static_cast<float*>(workspace);
  colsum_partial_kernel<<<(unsigned)nblk, 256, 0, st>>>(rows, (int32_t)F, x, ldx, rpb, part);
  GNN_LAUNCH_CHECK();
  colsum_final_kernel<<<(unsigned)F, 256, 0, st>>>((int32_t)F, (int32_t)nblk, part, out);
  GNN_LAUNCH_CHECK();
  return GNN_OK;
}
