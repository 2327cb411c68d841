// K12 — the per-layer tail of SAGEResBNNet (src/models/gnn.py:182-194), training mode:
//     h = dropout(relu(BatchNorm1d(z))) + r          r = res_proj(h_prev)
// replacing torch's batch_norm_collect_statistics / transform_input / backward_reduce /
// backward_elemt kernels, the ReLU, dropout and residual-add kernels and their backward passes
// (about a dozen ATen launches per layer, 5 of them full [N, C] passes over HBM) by:
//   forward : stats (one pass: per-block Σz, Σz² in float64) -> finalize (batch mean, invstd,
//             running-stat update; for SyncBN the caller all-reduces the [2C + 1] stats
//             between the two) -> apply (one fused elementwise pass)
//   backward: reduce (Σdy, Σdy·x̂ of the BN output gradient dy = dh ⊙ dropout ⊙ relu', dy
//             recomputed from z, per-block partials) -> merge -> apply (dz, one pass)
// Dropout is the counter hash of the fused SAGE path (keep_elem of element r·C + c; the mask is
// recomputed in the backward, oracle/dropout_hash.py reproduces it).  Reductions are
// fixed-order (per-block partials merged in block order): bitwise reproducible.
#include "common.hpp"
#include "gemm_common.hpp"  // keep_elem

namespace gnnmp {
namespace {

constexpr int kBnThreads = 256;
constexpr int kBnBlocks = 2048;  // per-block partials (rows split into <= 2048 contiguous ranges)
constexpr int kBnU = 8;          // rows in flight per thread in the reduction passes

struct BnArgs {
  const float* z; int64_t ldz;
  const float* r; int64_t ldr;
  const float* dh; int64_t lddh;
  float* out; int64_t ldo;
  int64_t N; int32_t C;
  const float* mean; const float* invstd; const float* weight; const float* bias;
  int32_t dropout; uint32_t keep_thresh; float drop_scale; uint64_t seed; const int64_t* seed_ptr;
};

__device__ __forceinline__ uint64_t bn_seed(const BnArgs& a) {
  return a.seed_ptr ? (uint64_t)(*a.seed_ptr) * 0x9E3779B97F4A7C15ull + a.seed : a.seed;
}

// Column-parallel block layout: cols = min(C, 256) columns x lanes = 256 / cols row lanes; a wave
// reads 64 consecutive columns of one row (coalesced).  Block b owns rows [b·R, (b+1)·R).
// stats: part[b][0][c] = Σ z, part[b][1][c] = Σ z² (float64: the one-pass variance stays exact to
// ~1e-16 relative even for features with a large mean).
__global__ __launch_bounds__(kBnThreads) void bn_stats_partial_kernel(BnArgs a, int64_t R, double* __restrict__ part) {
  __shared__ double red[2][kBnThreads];
  const int C = a.C;
  const int cols = C < kBnThreads ? C : kBnThreads;
  const int lanes = kBnThreads / cols;
  const int cl = threadIdx.x % cols, rl = threadIdx.x / cols;
  const int64_t r0 = blockIdx.x * R, r1 = min(a.N, r0 + R);
  for (int cb = 0; cb < C; cb += cols) {
    const int c = cb + cl;
    double s = 0.0, q = 0.0;
    if (rl < lanes && c < C) {
      // kBnU independent row loads in flight per thread, then the float64 sums in row order
      for (int64_t rb = r0 + rl; rb < r1; rb += (int64_t)kBnU * lanes) {
        float v[kBnU];
#pragma unroll
        for (int u = 0; u < kBnU; ++u) {
          const int64_t r = rb + (int64_t)u * lanes;
          v[u] = a.z[(r < r1 ? r : r0) * a.ldz + c];  // clamped, unconditional: the 8 loads stay in flight
        }
#pragma unroll
        for (int u = 0; u < kBnU; ++u)
          if (rb + (int64_t)u * lanes >= r1) v[u] = 0.0f;
#pragma unroll
        for (int u = 0; u < kBnU; ++u) {
          const double d = v[u];
          s += d;
          q = fma(d, d, q);
        }
      }
    }
    red[0][threadIdx.x] = s;
    red[1][threadIdx.x] = q;
    __syncthreads();
    if (threadIdx.x < cols && cb + (int)threadIdx.x < C) {
      double ss = 0.0, qq = 0.0;
      for (int l = 0; l < lanes; ++l) {
        ss += red[0][l * cols + threadIdx.x];
        qq += red[1][l * cols + threadIdx.x];
      }
      part[(int64_t)blockIdx.x * 2 * C + cb + threadIdx.x] = ss;
      part[(int64_t)blockIdx.x * 2 * C + C + cb + threadIdx.x] = qq;
    }
    __syncthreads();
  }
}

// stats[0..C) = Σz, stats[C..2C) = Σz², stats[2C] = n (float64; summable across ranks).
// With `fin`, also the finalize step below in the same launch (single device).
__device__ void bn_finalize_one(int c, const double* stats, int C, float eps, float momentum, float* mean,
                                float* invstd, float* rmean, float* rvar, const int64_t* nbt) {
  const double n = stats[2 * C];
  const double m = stats[c] / n;
  const double var = fmax(stats[C + c] / n - m * m, 0.0);
  mean[c] = (float)m;
  invstd[c] = 1.0f / sqrtf((float)var + eps);
  if (rmean) {  // nn.BatchNorm1d: momentum update with the unbiased variance
    const float mom = momentum >= 0.f ? momentum : 1.0f / (float)(*nbt + 1);  // None: cumulative average
    const float unb = (float)(var * (n / fmax(n - 1.0, 1.0)));
    rmean[c] = (1.0f - mom) * rmean[c] + mom * (float)m;
    rvar[c] = (1.0f - mom) * rvar[c] + mom * unb;
  }
}

// stats[v] = Σ_b part[b][v] for v < 2C (one block per v: threads stride the partials in a fixed
// order, then a fixed LDS tree), stats[2C] = N.
template <typename T, typename S>
__global__ __launch_bounds__(kBnThreads) void bn_merge_kernel(const T* __restrict__ part, int nblk, int C, int64_t N,
                                                              S* __restrict__ out) {
  __shared__ S red[kBnThreads];
  const int v = blockIdx.x;
  S acc = 0;
  for (int b = threadIdx.x; b < nblk; b += kBnThreads) acc += part[(int64_t)b * 2 * C + v];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int h = kBnThreads / 2; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[v] = red[0];
    if (N >= 0 && v == 0) out[2 * C] = (S)N;
  }
}

// Single device: the merge and the finalize in one launch — block c sums column c's Σz and Σz²
// partials (bn_merge_kernel's order and LDS tree, bit for bit) and finalizes column c itself (a
// column's mean / invstd / running stats need only its own two sums), so no block waits on another
// and the separate finalize launch is gone.  Block 0 bumps num_batches_tracked.  Taken for a fixed
// momentum only: the cumulative average (momentum None) reads num_batches_tracked in every column,
// which block 0's bump could not be ordered against; SyncBN keeps the separate finalize too (its
// stats are all-reduced in between).
__global__ __launch_bounds__(kBnThreads) void bn_merge_finalize_kernel(const double* __restrict__ part, int nblk, int C,
                                                                       int64_t N, double* __restrict__ stats, float eps,
                                                                       float momentum, float* mean, float* invstd,
                                                                       float* rmean, float* rvar, int64_t* nbt) {
  __shared__ double red[2][kBnThreads];
  const int c = blockIdx.x;
  double s = 0, q = 0;
  for (int b = threadIdx.x; b < nblk; b += kBnThreads) {
    s += part[(int64_t)b * 2 * C + c];
    q += part[(int64_t)b * 2 * C + C + c];
  }
  red[0][threadIdx.x] = s;
  red[1][threadIdx.x] = q;
  __syncthreads();
  for (int h = kBnThreads / 2; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) {
      red[0][threadIdx.x] += red[0][threadIdx.x + h];
      red[1][threadIdx.x] += red[1][threadIdx.x + h];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    stats[c] = red[0][0];
    stats[C + c] = red[1][0];
    stats[2 * C] = (double)N;  // (every block writes the same value)
    double loc[3];              // this column's sums and n, as bn_finalize_one reads them from stats
    loc[0] = red[0][0];
    loc[1] = red[1][0];
    loc[2] = (double)N;
    float m, is;
    float* rm = rmean ? rmean + c : nullptr;
    float* rv = rvar ? rvar + c : nullptr;
    bn_finalize_one(0, loc, 1, eps, momentum, &m, &is, rm, rv, nbt);
    mean[c] = m;
    invstd[c] = is;
    if (c == 0 && nbt) *nbt += 1;
  }
}

__global__ __launch_bounds__(kBnThreads) void bn_finalize_kernel(const double* __restrict__ stats, int C, float eps,
                                                                float momentum, float* mean, float* invstd, float* rmean,
                                                                float* rvar, int64_t* nbt) {
  for (int c = threadIdx.x; c < C; c += blockDim.x) bn_finalize_one(c, stats, C, eps, momentum, mean, invstd, rmean, rvar, nbt);
  __syncthreads();
  if (threadIdx.x == 0 && nbt) *nbt += 1;
}

// BN output y = (z - mean)·invstd·w + b of element (r, c)
__device__ __forceinline__ float bn_y(const BnArgs& a, float z, int c) {
  return (z - a.mean[c]) * a.invstd[c] * a.weight[c] + a.bias[c];
}

// forward apply: out = dropout(relu(y)) + r.  Threads as (column, row lane) like the reductions
// (no per-element division); blocks stride over row groups.  (r12: 4 rows in flight per thread,
// loads first, measured 28.8 -> 29.5 us here and 26.4 -> 29.9 us in the backward apply: kept 1.)
__global__ __launch_bounds__(kBnThreads) void bn_act_res_fwd_kernel(BnArgs a) {
  const uint64_t seed = a.dropout ? bn_seed(a) : 0;
  const int C = a.C;
  const int cols = C < kBnThreads ? C : kBnThreads;
  const int lanes = kBnThreads / cols;
  const int cl = threadIdx.x % cols, rl = threadIdx.x / cols;
  if (rl >= lanes) return;
  for (int cb = 0; cb < C; cb += cols) {
    const int c = cb + cl;
    if (c >= C) break;
    const float m = a.mean[c], is = a.invstd[c], w = a.weight[c], b = a.bias[c];
    for (int64_t r = (int64_t)blockIdx.x * lanes + rl; r < a.N; r += (int64_t)gridDim.x * lanes) {
      float y = fmaxf((a.z[r * a.ldz + c] - m) * is * w + b, 0.0f);
      if (a.dropout) y = keep_elem(seed, (uint32_t)(r * C + c), a.keep_thresh) ? y * a.drop_scale : 0.0f;
      a.out[r * a.ldo + c] = y + (a.r ? a.r[r * a.ldr + c] : 0.0f);
    }
  }
}

// dy = dh ⊙ keep·scale ⊙ [y > 0] and x̂ of element i
__device__ __forceinline__ void bn_dy(const BnArgs& a, uint64_t seed, int64_t r, int c, int64_t i, float& dy, float& xh) {
  const float z = a.z[r * a.ldz + c];
  xh = (z - a.mean[c]) * a.invstd[c];
  const float y = xh * a.weight[c] + a.bias[c];
  float g = a.dh[r * a.lddh + c];
  if (a.dropout) g = keep_elem(seed, (uint32_t)i, a.keep_thresh) ? g * a.drop_scale : 0.0f;
  dy = y > 0.0f ? g : 0.0f;
}

// backward reduce: part[b][0][c] = Σ dy, part[b][1][c] = Σ dy·x̂ over block b's rows
__global__ __launch_bounds__(kBnThreads) void bn_bwd_partial_kernel(BnArgs a, int64_t R, float* __restrict__ part) {
  __shared__ float red[2][kBnThreads];
  const uint64_t seed = a.dropout ? bn_seed(a) : 0;
  const int C = a.C;
  const int cols = C < kBnThreads ? C : kBnThreads;
  const int lanes = kBnThreads / cols;
  const int cl = threadIdx.x % cols, rl = threadIdx.x / cols;
  const int64_t r0 = blockIdx.x * R, r1 = min(a.N, r0 + R);
  for (int cb = 0; cb < C; cb += cols) {
    const int c = cb + cl;
    float s0 = 0.f, s1 = 0.f, q0 = 0.f, q1 = 0.f;  // two interleaved chains each
    if (rl < lanes && c < C) {
      for (int64_t rb = r0 + rl; rb < r1; rb += (int64_t)kBnU * lanes) {
        float dy[kBnU], xh[kBnU];
#pragma unroll
        for (int u = 0; u < kBnU; ++u) {
          const int64_t r = rb + (int64_t)u * lanes;
          const int64_t rr = r < r1 ? r : r0;  // rows past the block: loaded, then dropped
          bn_dy(a, seed, rr, c, rr * C + c, dy[u], xh[u]);
          if (r >= r1) dy[u] = 0.0f;
        }
#pragma unroll
        for (int u = 0; u < kBnU; u += 2) {
          s0 += dy[u]; q0 = fmaf(dy[u], xh[u], q0);
          s1 += dy[u + 1]; q1 = fmaf(dy[u + 1], xh[u + 1], q1);
        }
      }
    }
    red[0][threadIdx.x] = s0 + s1;
    red[1][threadIdx.x] = q0 + q1;
    __syncthreads();
    if (threadIdx.x < cols && cb + (int)threadIdx.x < C) {
      float ss = 0.f, qq = 0.f;
      for (int l = 0; l < lanes; ++l) {
        ss += red[0][l * cols + threadIdx.x];
        qq += red[1][l * cols + threadIdx.x];
      }
      part[(int64_t)blockIdx.x * 2 * C + cb + threadIdx.x] = ss;
      part[(int64_t)blockIdx.x * 2 * C + C + cb + threadIdx.x] = qq;
    }
    __syncthreads();
  }
}

// backward apply: dz = w·invstd·(dy − Σdy/n − x̂·Σdy·x̂/n)  (sums over every rank's rows)
// colsum (optional, C <= kBnThreads): the block's column sums of the dz it stores, colsum[b·C + c]
// (each thread's rows in order, the row lanes in order): the bias gradient of the conv below
// (SAGE-ResBN layer 0's transform-first conv) without a pass over dz
__global__ __launch_bounds__(kBnThreads) void bn_bwd_apply_kernel(BnArgs a, const float* __restrict__ sums,
                                                                 const double* __restrict__ n_total,
                                                                 float* __restrict__ colsum = nullptr) {
  __shared__ float csh[kBnThreads];
  const uint64_t seed = a.dropout ? bn_seed(a) : 0;
  const float inv_n = (float)(1.0 / *n_total);
  const int C = a.C;
  const int cols = C < kBnThreads ? C : kBnThreads;
  const int lanes = kBnThreads / cols;
  const int cl = threadIdx.x % cols, rl = threadIdx.x / cols;
  float cs = 0.f;
  for (int cb = 0; rl < lanes && cb < C; cb += cols) {
    const int c = cb + cl;
    if (c >= C) break;
    const float k = a.weight[c] * a.invstd[c], s0 = sums[c] * inv_n, s1 = sums[C + c] * inv_n;
    for (int64_t r = (int64_t)blockIdx.x * lanes + rl; r < a.N; r += (int64_t)gridDim.x * lanes) {
      float dy, xh;
      bn_dy(a, seed, r, c, r * C + c, dy, xh);
      const float v = k * (dy - s0 - xh * s1);
      a.out[r * a.ldo + c] = v;
      cs += v;
    }
  }
  if (!colsum) return;  // kernel-uniform (C <= kBnThreads: one column pass)
  csh[threadIdx.x] = rl < lanes ? cs : 0.f;
  __syncthreads();
  if (rl == 0) {
    float t = csh[cl];
    for (int l = 1; l < lanes; ++l) t += csh[l * cols + cl];
    colsum[(int64_t)blockIdx.x * C + cl] = t;
  }
}

// row-group blocks of the apply kernels: enough to fill the chip (8 blocks per CU), at most one
// row group per block and pass
unsigned bn_grid(int64_t N, int64_t C) {
  const int64_t lanes = C < kBnThreads ? kBnThreads / C : 1;
  const int64_t b = ceil_div(N, lanes);
  return (unsigned)(b < 2048 ? (b > 0 ? b : 1) : 2048);
}

// rows per reduction block: a multiple of (row lanes × kBnU), so every thread runs whole unrolled
// iterations (100-row blocks left 25 rows per thread = 3 full + 1 one-row iteration: r12 measured the
// backward partial 33.7 us before)
int64_t bn_rows_per_block(int64_t N, int64_t C) {
  const int64_t lanes = C < kBnThreads ? kBnThreads / C : 1;
  const int64_t unit = lanes * kBnU;
  return ceil_div(ceil_div(N, kBnBlocks), unit) * unit;
}

gnn_status bn_args(const char* fn, int64_t N, int64_t C, const float* mean, const float* invstd, const float* weight,
                   const float* bias, float dropout_p, uint64_t seed, const int64_t* seed_ptr, BnArgs& a) {
  if (N < 0 || C < 1 || C > 4096) return fail(GNN_ERR_INVALID_ARG, fn, "bad N / C");
  if (N * C >= ((int64_t)1 << 32)) return fail(GNN_ERR_UNSUPPORTED, fn, "N·C must be < 2^32 (dropout element index)");
  if (!mean || !invstd || !weight || !bias) return fail(GNN_ERR_INVALID_ARG, fn, "null BN parameters");
  if (dropout_p < 0.f || dropout_p >= 1.f) return fail(GNN_ERR_INVALID_ARG, fn, "dropout p in [0,1)");
  a.N = N; a.C = (int32_t)C;
  a.mean = mean; a.invstd = invstd; a.weight = weight; a.bias = bias;
  a.dropout = dropout_p > 0.f;
  a.keep_thresh = (uint32_t)((1.0 - (double)dropout_p) * 16777216.0);
  a.drop_scale = a.dropout ? (float)(1.0 / (1.0 - (double)dropout_p)) : 1.0f;
  a.seed = seed; a.seed_ptr = seed_ptr;
  return GNN_OK;
}

}  // namespace
}  // namespace gnnmp

using namespace gnnmp;

extern "C" gnn_status gnn_bn_workspace_size(int64_t C, size_t* bytes) {
  if (!bytes || C < 1) return fail(GNN_ERR_INVALID_ARG, __func__, "bad args");
  *bytes = (size_t)kBnBlocks * 2 * (size_t)C * sizeof(double);
  return GNN_OK;
}

extern "C" gnn_status gnn_bn_stats_f32(const float* z, int64_t ldz, int64_t N, int64_t C, double* stats, int32_t finalize,
                                       float eps, float momentum, float* mean, float* invstd, float* running_mean,
                                       float* running_var, int64_t* num_batches_tracked, void* workspace,
                                       size_t workspace_bytes, gnn_stream_t stream) {
  if (N < 1 || C < 1 || C > 4096 || ldz < C || !z || !stats) return fail(GNN_ERR_INVALID_ARG, __func__, "bad args");
  if (finalize && (!mean || !invstd || (running_mean && !running_var)))
    return fail(GNN_ERR_INVALID_ARG, __func__, "finalize needs mean / invstd (and running_var with running_mean)");
  if (!workspace || workspace_bytes < (size_t)kBnBlocks * 2 * (size_t)C * sizeof(double))
    return fail(GNN_ERR_WORKSPACE, __func__, "workspace too small");
  hipStream_t st = (hipStream_t)stream;
  BnArgs a{};
  a.z = z; a.ldz = ldz; a.N = N; a.C = (int32_t)C;
  const int64_t R = bn_rows_per_block(N, C);
  const int nblk = (int)ceil_div(N, R);
  double* part = static_cast<double*>(workspace);
  bn_stats_partial_kernel<<<nblk, kBnThreads, 0, st>>>(a, R, part);
  GNN_LAUNCH_CHECK();
  if (finalize && momentum >= 0.f) {
    bn_merge_finalize_kernel<<<(unsigned)C, kBnThreads, 0, st>>>(part, nblk, (int)C, N, stats, eps, momentum, mean,
                                                                 invstd, running_mean, running_var, num_batches_tracked);
    GNN_LAUNCH_CHECK();
    return GNN_OK;
  }
  bn_merge_kernel<double, double><<<(unsigned)(2 * C), kBnThreads, 0, st>>>(part, nblk, (int)C, N, stats);
  GNN_LAUNCH_CHECK();
  if (finalize) {
    bn_finalize_kernel<<<1, kBnThreads, 0, st>>>(stats, (int)C, eps, momentum, mean, invstd, running_mean, running_var,
                                                 num_batches_tracked);
    GNN_LAUNCH_CHECK();
  }
  return GNN_OK;
}

extern "C" gnn_status gnn_bn_finalize_f32(const double* stats, int64_t C, float eps, float momentum, float* mean,
                                          float* invstd, float* running_mean, float* running_var,
                                          int64_t* num_batches_tracked, gnn_stream_t stream) {
  if (!stats || C < 1 || C > 4096 || !mean || !invstd || (running_mean && !running_var))
    return fail(GNN_ERR_INVALID_ARG, __func__, "bad args");
  bn_finalize_kernel<<<1, kBnThreads, 0, (hipStream_t)stream>>>(stats, (int)C, eps, momentum, mean, invstd, running_mean,
                                                                running_var, num_batches_tracked);
  GNN_LAUNCH_CHECK();
  return GNN_OK;
}

extern "C" gnn_status gnn_bn_act_res_fwd_f32(const float* z, int64_t ldz, const float* r, int64_t ldr, int64_t N, int64_t C,
                                             const float* mean, const float* invstd, const float* weight,
                                             const float* bias, float dropout_p, uint64_t seed, const int64_t* seed_ptr,
                                             float* h, int64_t ldh, gnn_stream_t stream) {
  BnArgs a{};
  gnn_status s = bn_args(__func__, N, C, mean, invstd, weight, bias, dropout_p, seed, seed_ptr, a);
  if (s != GNN_OK) return s;
  if (!z || !h || ldz < C || ldh < C || (r && ldr < C)) return fail(GNN_ERR_INVALID_ARG, __func__, "bad z / r / h");
  if (N == 0) return GNN_OK;
  a.z = z; a.ldz = ldz; a.r = r; a.ldr = ldr; a.out = h; a.ldo = ldh;
  bn_act_res_fwd_kernel<<<bn_grid(N, C), kBnThreads, 0, (hipStream_t)stream>>>(a);
  GNN_LAUNCH_CHECK();
  return GNN_OK;
}

extern "C" gnn_status gnn_bn_act_bwd_reduce_f32(const float* dh, int64_t lddh, const float* z, int64_t ldz, int64_t N,
                                                int64_t C, const float* mean, const float* invstd, const float* weight,
                                                const float* bias, float dropout_p, uint64_t seed,
                                                const int64_t* seed_ptr, float* sums, void* workspace,
                                                size_t workspace_bytes, gnn_stream_t stream) {
  BnArgs a{};
  gnn_status s = bn_args(__func__, N, C, mean, invstd, weight, bias, dropout_p, seed, seed_ptr, a);
  if (s != GNN_OK) return s;
  if (!dh || !z || !sums || lddh < C || ldz < C) return fail(GNN_ERR_INVALID_ARG, __func__, "bad dh / z / sums");
  if (!workspace || workspace_bytes < (size_t)kBnBlocks * 2 * (size_t)C * sizeof(float))
    return fail(GNN_ERR_WORKSPACE, __func__, "workspace too small");
  hipStream_t st = (hipStream_t)stream;
  if (N == 0) return hip_check(hipMemsetAsync(sums, 0, 2 * C * sizeof(float), st), __func__);
  a.dh = dh; a.lddh = lddh; a.z = z; a.ldz = ldz;
  const int64_t R = bn_rows_per_block(N, C);
  const int nblk = (int)ceil_div(N, R);
  float* part = static_cast<float*>(workspace);
  bn_bwd_partial_kernel<<<nblk, kBnThreads, 0, st>>>(a, R, part);
  GNN_LAUNCH_CHECK();
  bn_merge_kernel<float, float><<<(unsigned)(2 * C), kBnThreads, 0, st>>>(part, nblk, (int)C, -1, sums);
  GNN_LAUNCH_CHECK();
  return GNN_OK;
}

extern "C" gnn_status gnn_bn_act_bwd_colsum_blocks(int64_t N, int64_t C, int32_t* nb) {
  if (!nb || N < 1 || C < 1) return fail(GNN_ERR_INVALID_ARG, __func__, "bad args");
  *nb = C <= kBnThreads ? (int32_t)bn_grid(N, C) : 0;
  return GNN_OK;
}

static gnn_status bn_act_bwd(const char* fn, const float* dh, int64_t lddh, const float* z, int64_t ldz, int64_t N,
                             int64_t C, const float* mean, const float* invstd, const float* weight, const float* bias,
                             float dropout_p, uint64_t seed, const int64_t* seed_ptr, const float* sums,
                             const double* n_total, float* dz, int64_t lddz, float* colsum, gnn_stream_t stream);

extern "C" gnn_status gnn_bn_act_bwd_colsum_f32(const float* dh, int64_t lddh, const float* z, int64_t ldz, int64_t N,
                                                int64_t C, const float* mean, const float* invstd, const float* weight,
                                                const float* bias, float dropout_p, uint64_t seed,
                                                const int64_t* seed_ptr, const float* sums, const double* n_total,
                                                float* dz, int64_t lddz, float* colsum, gnn_stream_t stream) {
  if (!colsum || C > kBnThreads || N < 1) return fail(GNN_ERR_INVALID_ARG, __func__, "colsum needs N >= 1, C <= 256");
  return bn_act_bwd(__func__, dh, lddh, z, ldz, N, C, mean, invstd, weight, bias, dropout_p, seed, seed_ptr, sums,
                    n_total, dz, lddz, colsum, stream);
}

extern "C" gnn_status gnn_bn_act_bwd_f32(const float* dh, int64_t lddh, const float* z, int64_t ldz, int64_t N, int64_t C,
                                         const float* mean, const float* invstd, const float* weight, const float* bias,
                                         float dropout_p, uint64_t seed, const int64_t* seed_ptr, const float* sums,
                                         const double* n_total, float* dz, int64_t lddz, gnn_stream_t stream) {
  return bn_act_bwd(__func__, dh, lddh, z, ldz, N, C, mean, invstd, weight, bias, dropout_p, seed, seed_ptr, sums,
                    n_total, dz, lddz, nullptr, stream);
}

static gnn_status bn_act_bwd(const char* fn, const float* dh, int64_t lddh, const float* z, int64_t ldz, int64_t N,
                             int64_t C, const float* mean, const float* invstd, const float* weight, const float* bias,
                             float dropout_p, uint64_t seed, const int64_t* seed_ptr, const float* sums,
                             const double* n_total, float* dz, int64_t lddz, float* colsum, gnn_stream_t stream) {
  const char* __func_name = fn;
  BnArgs a{};
  gnn_status s = bn_args(__func_name, N, C, mean, invstd, weight, bias, dropout_p, seed, seed_ptr, a);
  if (s != GNN_OK) return s;
  if (!dh || !z || !sums || !dz || !n_total || lddh < C || ldz < C || lddz < C)
    return fail(GNN_ERR_INVALID_ARG, __func_name, "bad dh / z / sums / dz / n");
  if (N == 0) return GNN_OK;
  a.dh = dh; a.lddh = lddh; a.z = z; a.ldz = ldz; a.out = dz; a.ldo = lddz;
  bn_bwd_apply_kernel<<<bn_grid(N, C), kBnThreads, 0, (hipStream_t)stream>>>(a, sums, n_total, colsum);
  return hip_check(hipGetLastError(), __func_name);
}

// ---- K13: SAGEResBNNet's input h0 = [x | sinusoid(t)] (src/models/gnn.py:145-160 the fixed
// sin/cos time features, :172-176 the concatenation), written in one pass.  torch runs it as ~10
// launches (long add, clamp, cast, reciprocal-multiply, arange, two muls, sin, cos, two cats), the
// last a full [N, F + dim] copy.  Same float32 operation order as torch's: t = (float)clamp(t-1) ·
// (1 / (T - 1)), freq_k = (float)k · (float)2π, sin / cos of t · freq_k.
namespace gnnmp {
namespace {

// Two rows per wave, lanes over columns, 256 columns per pass: all 8 loads of a pass issue before
// any store (clamped unconditional loads: no per-element branch, no 64-bit division).  Measured: a
// wave-per-row load→store loop 83 us, one thread per element with a 64-bit row division 145 us.
__global__ __launch_bounds__(256) void time_inject_sin_kernel(const float* __restrict__ x, int64_t ldx, int64_t N,
                                                              int F, const int64_t* __restrict__ t, int dim, int T,
                                                              float inv, float* __restrict__ out, int64_t ldo) {
  constexpr int R = 2, C = 4;
  const int lane = threadIdx.x & 63;
  const int64_t r0 = (((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6) * R;
  if (r0 >= N) return;
  const int W = F + dim;
  const int half = dim / 2;
  constexpr float kTwoPi = 6.283185307179586f;
  float tt[R];
  int64_t rr[R];
#pragma unroll
  for (int j = 0; j < R; ++j) {
    rr[j] = r0 + j < N ? r0 + j : r0;
    int64_t tc = t[rr[j]] - 1;
    tc = tc < 0 ? 0 : (tc > T - 1 ? T - 1 : tc);
    tt[j] = (float)tc * inv;
  }
  for (int c0 = 0; c0 < W; c0 += 64 * C) {
    float v[R][C];
#pragma unroll
    for (int j = 0; j < R; ++j)
#pragma unroll
      for (int i = 0; i < C; ++i) {
        const int c = c0 + lane + 64 * i;
        v[j][i] = x[rr[j] * ldx + (c < F ? c : F - 1)];
      }
#pragma unroll
    for (int j = 0; j < R; ++j) {
      if (r0 + j >= N) break;
#pragma unroll
      for (int i = 0; i < C; ++i) {
        const int c = c0 + lane + 64 * i;
        if (c >= W) break;
        float o = v[j][i];
        if (c >= F) {
          const int k = c - F;
          if (k < half) o = sinf(tt[j] * ((float)(k + 1) * kTwoPi));
          else if (k < 2 * half) o = cosf(tt[j] * ((float)(k - half + 1) * kTwoPi));
          else o = 0.0f;
        }
        out[rr[j] * ldo + c] = o;
      }
    }
  }
}

}  // namespace
}  // namespace gnnmp

using namespace gnnmp;

extern "C" gnn_status gnn_time_inject_sin_f32(const float* x, int64_t ldx, int64_t N, int64_t F, const int64_t* t_idx,
                                              int64_t dim, int64_t max_timestep, float* out, int64_t ldo,
                                              gnn_stream_t stream) {
  if (N < 0 || F < 1 || dim < 1 || max_timestep < 1 || F + dim > (1 << 20) || ldx < F || ldo < F + dim ||
      (N > 0 && (!x || !t_idx || !out)))
    return fail(GNN_ERR_INVALID_ARG, __func__, "bad args");
  if (N == 0) return GNN_OK;
  const float inv = 1.0f / (float)(max_timestep - 1 > 1 ? max_timestep - 1 : 1);
  time_inject_sin_kernel<<<(unsigned)ceil_div(N, 4 * 2), 256, 0, (hipStream_t)stream>>>(
      x, ldx, N, (int)F, t_idx, (int)dim, (int)max_timestep, inv, out, ldo);
  GNN_LAUNCH_CHECK();
  return GNN_OK;
}
