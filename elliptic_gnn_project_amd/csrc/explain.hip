// Explain-mode edge scores: the gradient of a per-edge message multiplier.
//
// PyG 2.5.3 MessagePassing.propagate, with `explain` on, multiplies every message by
// edge_mask[e] (sigmoid applied by the caller) before the aggregation; GNNExplainer then
// optimises the mask (src/analysis/explain.py:593-672 drives it).  For SAGEConv's mean,
// out_i = (sum_e m_e x_j) / max(deg_i, 1), so d m_e = <dOut_i, x_j> / max(deg_i, 1): a sampled
// dense-dense product over the CSR slots.  The forward and the x-gradient reuse the EDGE_W
// aggregation (K5/K6's alpha-weighted form) with the mask as the slot weight.
//
// One wavefront per CSR row: dOut_i stays in L1/L2 across its slots, each slot's x_j row is
// read once with coalesced loads (lane f, f+64, ...), the dot reduces by xor shuffles, and
// lane 0 writes the slot's score to its PyG edge id (csr_eid), so the output is in edge order.
#include <hip/hip_runtime.h>

#include "common.hpp"

using namespace gnnmp;

namespace {

constexpr int kWavesPerBlock = 4;

__global__ void __launch_bounds__(64 * kWavesPerBlock)
edge_dot_kernel(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                const int32_t* __restrict__ eid, const float* __restrict__ nodew,
                const float* __restrict__ a, int64_t lda, const float* __restrict__ b, int64_t ldb,
                int32_t F, int64_t N, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  if (r >= N) return;
  const float d = nodew ? fmaxf(nodew[r], 1.0f) : 1.0f;
  const float* ar = a + r * lda;
  const int32_t s1 = rowptr[r + 1];
  for (int32_t s = rowptr[r]; s < s1; ++s) {
    const float* bj = b + (int64_t)col[s] * ldb;
    float acc = 0.0f;
    for (int f = lane; f < F; f += 64) acc = fmaf(ar[f], bj[f], acc);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (lane == 0) out[eid ? (int64_t)eid[s] : (int64_t)s] = acc / d;
  }
}

}  // namespace

extern "C" gnn_status gnn_edge_dot_f32(const gnn_graph* g, const int32_t* eid, const float* nodew,
                                       const float* a, int64_t lda, const float* b, int64_t ldb,
                                       int64_t F, float* out, gnn_stream_t stream) {
  if (!g || !out || (F > 0 && (!a || !b)) || F < 0 || F > INT32_MAX || lda < F || ldb < F)
    return fail(GNN_ERR_INVALID_ARG, __func__, "null pointer or bad width/leading dimension");
  const int64_t N = g->num_nodes;
  if (N == 0 || g->num_slots == 0) return GNN_OK;
  if (!g->rowptr || !g->col) return fail(GNN_ERR_INVALID_ARG, __func__, "graph without CSR");
  const int64_t blocks = (N + kWavesPerBlock - 1) / kWavesPerBlock;
  hipLaunchKernelGGL(edge_dot_kernel, dim3((unsigned)blocks), dim3(64 * kWavesPerBlock), 0,
                     (hipStream_t)stream, g->rowptr, g->col, eid, nodew, a, lda, b, ldb, (int32_t)F, N,
                     out);
  return hip_check(hipGetLastError(), __func__);
}
