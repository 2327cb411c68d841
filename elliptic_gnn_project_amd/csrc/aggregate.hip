// K1 / K2 / K4 — atomic-free segmented aggregation over a graph plan (fp32).
//
// Replaces PyG 2.5.3 MessagePassing.propagate for:
//   SAGEConv  (aggr='mean'):   x_j = x.index_select(0, ei[0]); scatter(x_j, ei[1], reduce='mean')
//             = zeros.scatter_add_(x_j) / count.clamp(min=1)          (src/models/gnn.py:49,52,187,193)
//   its backward: grad/count then index_add over ei[0]               (the CSC "MEAN_BWD" mode)
//   GCNConv:  message edge_weight * x_j, aggr='add', edge_weight = dinv[j]*dinv[i]  (gnn.py:28,31)
//   GATConv:  message alpha * x_j per head (gnn.py:72,75)
//
// Mapping (CDNA4): one wave64 per destination row; the row's slot range and neighbour
// ids are wave-uniform (scalar loads); lanes stride the F features with VEC-wide
// (float2/float4) loads so each gathered row is read as contiguous 256-1024 B
// wave-instructions.  Slots are summed in plan order (PyG edge order) with one
// accumulator per feature: no atomics, bitwise reproducible.  Loads of up to 4
// neighbours are issued before their adds to keep several rows in flight per wave.
// Rows with F <= 8 (e.g. 2-class logits) use one lane per row instead.
#include "common.hpp"

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
  const float* bias;
  int32_t relu;
  int64_t nrows;
  int32_t F;
};

// Per-slot scaled contribution.
template <int MODE, int VEC>
__device__ __forceinline__ void contrib(const AggArgs& a, int32_t n, int32_t r, int64_t slot,
                                        int f0, float (&v)[VEC]) {
  if constexpr (MODE == GNN_AGG_MEAN_BWD) {
    float d = fmaxf(a.nodew[n], 1.0f);
#pragma unroll
    for (int q = 0; q < VEC; ++q) v[q] = v[q] / d;
  } else if constexpr (MODE == GNN_AGG_GCN) {
    float w = a.nodew[n] * a.nodew[r];
#pragma unroll
    for (int q = 0; q < VEC; ++q) v[q] = w * v[q];
  } else if constexpr (MODE == GNN_AGG_EDGE_W) {
    int64_t ws = a.wslot ? (int64_t)a.wslot[slot] : slot;
    float w = a.ew[ws * a.heads + f0 / a.chan];
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
  if (a.bias) {
#pragma unroll
    for (int q = 0; q < VEC; ++q) acc[q] += a.bias[f0 + q];
  }
  if (a.relu) {
#pragma unroll
    for (int q = 0; q < VEC; ++q) acc[q] = fmaxf(acc[q], 0.0f);
  }
}

// One wave per row; 4 waves per 256-thread block; grid-stride over rows.
template <int MODE, int VEC>
__global__ __launch_bounds__(256) void agg_rowwave_kernel(AggArgs a) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int nchunk = a.F / VEC;
  for (int64_t r = (int64_t)blockIdx.x * 4 + wave; r < a.nrows; r += (int64_t)gridDim.x * 4) {
    const int32_t beg = __builtin_amdgcn_readfirstlane(a.ptr[r]);
    const int32_t end = __builtin_amdgcn_readfirstlane(a.ptr[r + 1]);
    for (int c = lane; c < nchunk; c += 64) {
      const int f0 = c * VEC;
      float acc[VEC];
#pragma unroll
      for (int q = 0; q < VEC; ++q) acc[q] = 0.0f;
      int32_t k = beg;
      for (; k + 4 <= end; k += 4) {
        int32_t n0 = a.nbr[k], n1 = a.nbr[k + 1], n2 = a.nbr[k + 2], n3 = a.nbr[k + 3];
        float v0[VEC], v1[VEC], v2[VEC], v3[VEC];
        vload<VEC>(a.x + (int64_t)n0 * a.ldx + f0, v0);
        vload<VEC>(a.x + (int64_t)n1 * a.ldx + f0, v1);
        vload<VEC>(a.x + (int64_t)n2 * a.ldx + f0, v2);
        vload<VEC>(a.x + (int64_t)n3 * a.ldx + f0, v3);
        contrib<MODE, VEC>(a, n0, (int32_t)r, k, f0, v0);
        contrib<MODE, VEC>(a, n1, (int32_t)r, k + 1, f0, v1);
        contrib<MODE, VEC>(a, n2, (int32_t)r, k + 2, f0, v2);
        contrib<MODE, VEC>(a, n3, (int32_t)r, k + 3, f0, v3);
#pragma unroll
        for (int q = 0; q < VEC; ++q) acc[q] = (((acc[q] + v0[q]) + v1[q]) + v2[q]) + v3[q];
      }
      for (; k < end; ++k) {
        int32_t n = a.nbr[k];
        float v[VEC];
        vload<VEC>(a.x + (int64_t)n * a.ldx + f0, v);
        contrib<MODE, VEC>(a, n, (int32_t)r, k, f0, v);
#pragma unroll
        for (int q = 0; q < VEC; ++q) acc[q] += v[q];
      }
      finish<MODE, VEC>(a, r, f0, acc);
      vstore<VEC>(a.y + r * a.ldy + f0, acc);
    }
  }
}

// Narrow rows (F <= 8, e.g. 2-class logits): a group of 8 lanes per row, lanes over the
// row's slots (hubs are shared by 8 lanes), then a 3-step xor-shuffle reduction.
constexpr int kGroup = 8;
template <int MODE>
__global__ __launch_bounds__(256) void agg_group_kernel(AggArgs a) {
  const int sub = threadIdx.x & (kGroup - 1);
  for (int64_t r = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / kGroup; r < a.nrows;
       r += (int64_t)gridDim.x * blockDim.x / kGroup) {
    const int32_t beg = a.ptr[r];
    const int32_t end = a.ptr[r + 1];
    float acc[8];
#pragma unroll
    for (int f = 0; f < 8; ++f) acc[f] = 0.0f;
    for (int32_t k = beg + sub; k < end; k += kGroup) {
      const int32_t n = a.nbr[k];
      const float* xr = a.x + (int64_t)n * a.ldx;
#pragma unroll
      for (int f = 0; f < 8; ++f) {
        if (f < a.F) {
          float v[1] = {xr[f]};
          contrib<MODE, 1>(a, n, (int32_t)r, k, f, v);
          acc[f] += v[0];
        }
      }
    }
#pragma unroll
    for (int f = 0; f < 8; ++f) {
      if (f < a.F) {
#pragma unroll
        for (int off = kGroup / 2; off >= 1; off >>= 1) acc[f] += __shfl_xor(acc[f], off);
      }
    }
    if (sub == 0) {
#pragma unroll
      for (int f = 0; f < 8; ++f) {
        if (f < a.F) {
          float t[1] = {acc[f]};
          finish<MODE, 1>(a, r, f, t);
          a.y[r * a.ldy + f] = t[0];
        }
      }
    }
  }
}

bool aligned(const void* p, int bytes) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) % bytes) == 0; }

template <int MODE>
gnn_status launch_mode(const AggArgs& a, int vec, hipStream_t st) {
  if (a.nrows == 0 || a.F == 0) return GNN_OK;
  if (a.F <= 8) {
    int64_t blocks = ceil_div(a.nrows * kGroup, 256);
    if (blocks > ((int64_t)1 << 20)) blocks = (int64_t)1 << 20;
    agg_group_kernel<MODE><<<(unsigned)blocks, 256, 0, st>>>(a);
  } else {
    int64_t blocks = ceil_div(a.nrows, 4);
    if (blocks > (int64_t)1 << 20) blocks = (int64_t)1 << 20;
    if (vec == 4) agg_rowwave_kernel<MODE, 4><<<(unsigned)blocks, 256, 0, st>>>(a);
    else if (vec == 2) agg_rowwave_kernel<MODE, 2><<<(unsigned)blocks, 256, 0, st>>>(a);
    else agg_rowwave_kernel<MODE, 1><<<(unsigned)blocks, 256, 0, st>>>(a);
  }
  return hip_check(hipGetLastError(), "gnn_aggregate_f32");
}

// ------------------------------------------------------------------ colsum
// Stage 1: block b sums rows [b*rpb, (b+1)*rpb); threads form (row lanes x columns) so that
// narrow F still uses the whole block; row-lane partials are combined in LDS in fixed order.
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
    float acc = 0.0f;
    if (rl < lanes && c < F)
      for (int64_t r = r0 + rl; r < r1; r += lanes) acc += x[r * ldx + c];
    red[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x < cols && cb + (int)threadIdx.x < F) {
      float s = 0.0f;
      for (int l = 0; l < lanes; ++l) s += red[l * cols + threadIdx.x];
      part[(int64_t)blockIdx.x * F + cb + threadIdx.x] = s;
    }
    __syncthreads();
  }
}

__global__ void colsum_final_kernel(int32_t F, int32_t nblk, const float* __restrict__ part,
                                    float* __restrict__ out) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= F) return;
  float acc = 0.0f;
  for (int b = 0; b < nblk; ++b) acc += part[(int64_t)b * F + c];
  out[c] = acc;
}

constexpr int64_t kColsumBlocks = 256;

}  // namespace
}  // namespace gnnmp

using namespace gnnmp;

extern "C" gnn_status gnn_aggregate_f32(const gnn_graph* g, const gnn_agg_params* p, const float* x,
                                        int64_t ldx, int64_t F, float* y, int64_t ldy,
                                        gnn_stream_t stream) {
  if (!g || !p) return fail(GNN_ERR_INVALID_ARG, __func__, "null graph or params");
  if (F < 0 || F > INT32_MAX || ldx < F || ldy < F)
    return fail(GNN_ERR_INVALID_ARG, __func__, "bad F / leading dimensions");
  if (g->num_nodes > 0 && F > 0 && (!x || !y)) return fail(GNN_ERR_INVALID_ARG, __func__, "null x/y");
  if (p->addend && p->ld_add < F) return fail(GNN_ERR_INVALID_ARG, __func__, "bad ld_add");
  AggArgs a{};
  a.ptr = p->transpose ? g->colptr : g->rowptr;
  a.nbr = p->transpose ? g->row : g->col;
  a.wslot = (p->mode == GNN_AGG_EDGE_W && p->transpose) ? g->csc2csr : nullptr;
  a.nodew = p->nodew;
  a.ew = p->ew;
  a.heads = p->heads > 0 ? p->heads : 1;
  a.x = x; a.ldx = ldx; a.y = y; a.ldy = ldy;
  a.add = p->addend; a.ld_add = p->ld_add;
  a.bias = p->bias; a.relu = p->relu;
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
    if (p->mode == GNN_AGG_EDGE_W && a.chan % v) return false;
    int b = 4 * v;
    return aligned(x, b) && aligned(y, b) && aligned(p->addend, b);
  };
  int vec = ok_vec(4) ? 4 : (ok_vec(2) ? 2 : 1);
  hipStream_t st = (hipStream_t)stream;
  switch (p->mode) {
    case GNN_AGG_SUM: return launch_mode<GNN_AGG_SUM>(a, vec, st);
    case GNN_AGG_MEAN: return launch_mode<GNN_AGG_MEAN>(a, vec, st);
    case GNN_AGG_MEAN_BWD: return launch_mode<GNN_AGG_MEAN_BWD>(a, vec, st);
    case GNN_AGG_GCN: return launch_mode<GNN_AGG_GCN>(a, vec, st);
    case GNN_AGG_EDGE_W: return launch_mode<GNN_AGG_EDGE_W>(a, vec, st);
  }
  return fail(GNN_ERR_INVALID_ARG, __func__, "unknown mode");
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
  colsum_final_kernel<<<(unsigned)ceil_div(F, 64), 64, 0, st>>>((int32_t)F, (int32_t)nblk, part, out);
  GNN_LAUNCH_CHECK();
  return GNN_OK;
}
