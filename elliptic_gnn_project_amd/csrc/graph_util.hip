// Degree / GCN normalisation over a plan, and the library's status plumbing.
//
// gnn_in_degree_f32: PyG SAGEConv mean `count = scatter_add(ones, ei[1]).clamp(min=1)` keeps the
//   unclamped count here; the clamp happens inside the aggregation (GNN_AGG_MEAN*).
// gnn_gcn_norm_f32: PyG gcn_norm (add_remaining_self_loops already applied by the
//   GNN_LOOPS_REPLACE plan): deg = scatter_add(ones, col); dinv = deg.pow_(-0.5); inf -> 0.
//   Used by GCNConv at src/models/gnn.py:28,31.
#include <mutex>
#include <string>

#include "common.hpp"

namespace gnnmp {

namespace {
thread_local std::string g_last_error;

__global__ void in_degree_kernel(const int32_t* __restrict__ ptr, int64_t N, float* __restrict__ deg) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= N) return;
  deg[i] = (float)(ptr[i + 1] - ptr[i]);
}

__global__ void gcn_norm_kernel(const int32_t* __restrict__ ptr, int64_t N, float* __restrict__ dinv) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= N) return;
  float d = (float)(ptr[i + 1] - ptr[i]);
  float v = 1.0f / sqrtf(d);  // ATen pow(-0.5) == 1 / sqrt (correctly rounded ops)
  dinv[i] = isinf(v) ? 0.0f : v;
}
}  // namespace

void set_last_error(const std::string& msg) { g_last_error = msg; }

}  // namespace gnnmp

using namespace gnnmp;

extern "C" int gnn_abi_version(void) { return GNNMP_ABI_VERSION; }

extern "C" const char* gnn_status_string(gnn_status s) {
  switch (s) {
    case GNN_OK: return "ok";
    case GNN_ERR_INVALID_ARG: return "invalid argument";
    case GNN_ERR_INDEX_OUT_OF_RANGE: return "index out of range";
    case GNN_ERR_HIP: return "HIP runtime error";
    case GNN_ERR_WORKSPACE: return "workspace too small";
    case GNN_ERR_UNSUPPORTED: return "unsupported configuration";
  }
  return "unknown status";
}

extern "C" const char* gnn_last_error(void) { return g_last_error.c_str(); }

extern "C" gnn_status gnn_in_degree_f32(const gnn_graph* g, float* deg, gnn_stream_t stream) {
  if (!g || (g->num_nodes > 0 && (!deg || !g->rowptr))) return fail(GNN_ERR_INVALID_ARG, __func__, "null");
  if (g->num_nodes == 0) return GNN_OK;
  in_degree_kernel<<<(unsigned)ceil_div(g->num_nodes, 256), 256, 0, (hipStream_t)stream>>>(g->rowptr,
                                                                                          g->num_nodes, deg);
  GNN_LAUNCH_CHECK();
  return GNN_OK;
}

extern "C" gnn_status gnn_gcn_norm_f32(const gnn_graph* g, float* dinv, gnn_stream_t stream) {
  if (!g || (g->num_nodes > 0 && (!dinv || !g->rowptr))) return fail(GNN_ERR_INVALID_ARG, __func__, "null");
  if (g->num_nodes == 0) return GNN_OK;
  gcn_norm_kernel<<<(unsigned)ceil_div(g->num_nodes, 256), 256, 0, (hipStream_t)stream>>>(g->rowptr,
                                                                                         g->num_nodes, dinv);
  GNN_LAUNCH_CHECK();
  return GNN_OK;
}
