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
#include "common.hpp"

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
constexpr int kAttBlocks = 512;
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
  auto p3 = c.template take<float>((size_t)kAttBlocks * 2 * H * C_);
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
  gat_fwd_kernel<<<row_blocks(a.N), 256, 0, st>>>(a);
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
