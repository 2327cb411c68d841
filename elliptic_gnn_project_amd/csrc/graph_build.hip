// K0 — graph plan build: stable CSR-by-target and CSC-by-source from PyG edge_index.
//
// Replaces the per-call index handling PyG 2.5.3 does inside MessagePassing.propagate
// (index_select on edge_index[0], scatter on edge_index[1]) and, for GCN/GAT,
// torch_geometric.utils.{add_remaining_self_loops, remove_self_loops, add_self_loops}.
// The reference builds edge_index at src/train_gnn.py:320-324 (symmetrize by concat,
// no dedup) and passes it to every conv call (src/models/gnn.py:28,49,72,187).
//
// Ordering contract: within each CSR row (and CSC column) slots appear in PyG edge
// order, and the REPLACE-mode self loop is last, exactly where PyG's concatenation
// (edges..., arange(N) loops) puts it.  A stable LSD radix sort (rocPRIM onesweep)
// of (key, edge id) gives that order; all other passes are one thread per edge/node.
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>

#include "common.hpp"

namespace gnnmp {
namespace {

__global__ void prep_keys_kernel(const int64_t* __restrict__ ei, int64_t E, int64_t N, int replace,
                                 int32_t* __restrict__ key_dst, int32_t* __restrict__ key_src,
                                 int32_t* __restrict__ vals, int32_t* __restrict__ stats) {
  int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (e >= E) return;
  int64_t s = ei[e];
  int64_t d = ei[E + e];
  bool bad = (s < 0) | (s >= N) | (d < 0) | (d >= N);
  bool loop = !bad && (s == d);
  if (bad) atomicAdd(&stats[2], 1);
  if (loop) atomicAdd(&stats[1], 1);
  bool drop = bad || (replace && loop);
  key_dst[e] = drop ? (int32_t)N : (int32_t)d;
  key_src[e] = drop ? (int32_t)N : (int32_t)s;
  vals[e] = (int32_t)e;
}

// ptr[i] = first t with key[t] >= i, i in [0, N]; keys sorted, values in [0, N].
__global__ void boundaries_kernel(const int32_t* __restrict__ key, int64_t E, int64_t N,
                                  int32_t* __restrict__ ptr) {
  int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t > E) return;
  int64_t prev = (t == 0) ? -1 : key[t - 1];
  int64_t cur = (t == E) ? N : key[t];
  if (t == E) cur = N;  // fill the tail up to ptr[N]
  for (int64_t i = prev + 1; i <= cur && i <= N; ++i) ptr[i] = (int32_t)t;
}

__global__ void finish_ptr_kernel(const int32_t* __restrict__ nl_ptr, int64_t N, int replace,
                                  int32_t* __restrict__ ptr) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i > N) return;
  ptr[i] = nl_ptr[i] + (replace ? (int32_t)i : 0);
}

// One sorted edge -> its slot.  `other` is the endpoint stored in the slot.
__global__ void fill_slots_kernel(const int32_t* __restrict__ key_sorted,
                                  const int32_t* __restrict__ val_sorted, const int64_t* __restrict__ other,
                                  int64_t E, int64_t N, int replace, int32_t* __restrict__ nbr,
                                  int32_t* __restrict__ eid_out, int32_t* __restrict__ pos) {
  int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= E) return;
  int32_t i = key_sorted[t];
  if (i >= N) return;  // dropped (loop in REPLACE mode, or bad index)
  int32_t e = val_sorted[t];
  int64_t slot = t + (replace ? (int64_t)i : 0);
  nbr[slot] = (int32_t)other[e];
  eid_out[slot] = e;
  if (pos) pos[e] = (int32_t)slot;
}

__global__ void fill_loops_kernel(const int32_t* __restrict__ ptr, int64_t E, int64_t N,
                                  int32_t* __restrict__ nbr, int32_t* __restrict__ eid_out,
                                  int32_t* __restrict__ pos) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= N) return;
  int64_t slot = ptr[i + 1] - 1;
  nbr[slot] = (int32_t)i;
  eid_out[slot] = (int32_t)(E + i);
  if (pos) pos[E + i] = (int32_t)slot;
}

__global__ void csc2csr_kernel(const int32_t* __restrict__ colptr, int64_t N, int64_t Smax,
                               const int32_t* __restrict__ csc_eid, const int32_t* __restrict__ pos,
                               int32_t* __restrict__ csc2csr, int32_t* __restrict__ stats) {
  int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  int32_t S = colptr[N];
  if (t == 0) stats[0] = S;
  if (t >= Smax || t >= S) return;
  csc2csr[t] = pos[csc_eid[t]];
}

unsigned bits_for(int64_t v) {  // bits needed to hold values 0..v
  unsigned b = 1;
  while (b < 32 && (int64_t(1) << b) <= v) ++b;
  return b;
}

gnn_status sort_temp_bytes(int64_t E, size_t* bytes) {
  size_t tb = 0;
  hipError_t err = rocprim::radix_sort_pairs(nullptr, tb, (int32_t*)nullptr, (int32_t*)nullptr,
                                             (int32_t*)nullptr, (int32_t*)nullptr,
                                             (size_t)(E > 0 ? E : 1), 0, 32, (hipStream_t)0);
  if (err != hipSuccess) return hip_check(err, "sort_temp_bytes");
  *bytes = tb;
  return GNN_OK;
}

struct BuildLayout {
  int32_t *key_dst, *key_src, *vals, *key_out, *val_out, *nl_ptr, *pos, *csc_eid;
  void* sort_tmp;
  size_t sort_bytes;
};

template <typename Carver>
void carve(Carver& c, int64_t N, int64_t E, size_t sort_bytes, BuildLayout* L) {
  size_t e1 = (size_t)(E > 0 ? E : 1);
  size_t en = (size_t)(E + N + 1);
  auto k1 = c.template take<int32_t>(e1);
  auto k2 = c.template take<int32_t>(e1);
  auto v = c.template take<int32_t>(e1);
  auto ko = c.template take<int32_t>(e1);
  auto vo = c.template take<int32_t>(e1);
  auto np = c.template take<int32_t>((size_t)N + 1);
  auto ps = c.template take<int32_t>(en);
  auto ce = c.template take<int32_t>(en);
  auto st = c.template take<char>(sort_bytes);
  if (L) {
    L->key_dst = (int32_t*)k1; L->key_src = (int32_t*)k2; L->vals = (int32_t*)v;
    L->key_out = (int32_t*)ko; L->val_out = (int32_t*)vo; L->nl_ptr = (int32_t*)np;
    L->pos = (int32_t*)ps; L->csc_eid = (int32_t*)ce; L->sort_tmp = (void*)st;
    L->sort_bytes = sort_bytes;
  }
}

struct SizerAdapter {  // WorkspaceSizer returns void from take(); adapt to pointer-returning form
  WorkspaceSizer s;
  template <typename T>
  T* take(size_t n) { s.take<T>(n); return nullptr; }
};

}  // namespace
}  // namespace gnnmp

using namespace gnnmp;

extern "C" gnn_status gnn_graph_workspace_size(int64_t num_nodes, int64_t num_edges, size_t* bytes) {
  if (!bytes || num_nodes < 0 || num_edges < 0)
    return fail(GNN_ERR_INVALID_ARG, __func__, "negative size or null output");
  if (num_nodes >= INT32_MAX || num_edges + num_nodes >= INT32_MAX)
    return fail(GNN_ERR_INVALID_ARG, __func__, "N or E+N exceeds int32 range");
  size_t sb = 0;
  gnn_status s = sort_temp_bytes(num_edges, &sb);
  if (s != GNN_OK) return s;
  SizerAdapter a;
  carve(a, num_nodes, num_edges, sb, nullptr);
  *bytes = a.s.used + 256;
  return GNN_OK;
}

extern "C" gnn_status gnn_graph_build(const int64_t* edge_index, int64_t E, int64_t N,
                                      gnn_loop_mode loops, int32_t* rowptr, int32_t* col,
                                      int32_t* csr_eid, int32_t* colptr, int32_t* row,
                                      int32_t* csc2csr, int32_t* stats, void* workspace,
                                      size_t workspace_bytes, gnn_stream_t stream) {
  if (N < 0 || E < 0) return fail(GNN_ERR_INVALID_ARG, __func__, "negative N or E");
  if (N >= INT32_MAX || E + N >= INT32_MAX)
    return fail(GNN_ERR_INVALID_ARG, __func__, "N or E+N exceeds int32 range");
  if (!rowptr || !colptr || !stats || (E > 0 && (!edge_index || !col || !csr_eid || !row || !csc2csr)))
    return fail(GNN_ERR_INVALID_ARG, __func__, "null buffer");
  if (loops != GNN_LOOPS_KEEP && loops != GNN_LOOPS_REPLACE)
    return fail(GNN_ERR_INVALID_ARG, __func__, "unknown loop mode");
  const int replace = (loops == GNN_LOOPS_REPLACE);
  if (replace && N > 0 && (!col || !csr_eid || !row || !csc2csr))
    return fail(GNN_ERR_INVALID_ARG, __func__, "null buffer");
  hipStream_t st = (hipStream_t)stream;

  size_t sb = 0;
  gnn_status s = sort_temp_bytes(E, &sb);
  if (s != GNN_OK) return s;
  WorkspaceCarver c(workspace, workspace_bytes);
  BuildLayout L;
  carve(c, N, E, sb, &L);
  if (!c.ok) return fail(GNN_ERR_WORKSPACE, __func__, "workspace too small");

  GNN_HIP_TRY(hipMemsetAsync(stats, 0, 4 * sizeof(int32_t), st));
  const int TB = 256;
  const int64_t Smax = E + (replace ? N : 0);
  const unsigned bits = bits_for(N);
  const int64_t* src = edge_index;
  const int64_t* dst = edge_index + E;

  if (E > 0) {
    prep_keys_kernel<<<ceil_div(E, TB), TB, 0, st>>>(edge_index, E, N, replace, L.key_dst,
                                                     L.key_src, L.vals, stats);
    GNN_LAUNCH_CHECK();
  }
  // ---- CSR by target ----
  if (E > 0) {
    size_t tb = L.sort_bytes;
    GNN_HIP_TRY(rocprim::radix_sort_pairs(L.sort_tmp, tb, L.key_dst, L.key_out, L.vals, L.val_out,
                                          (size_t)E, 0, bits, st));
  }
  boundaries_kernel<<<ceil_div(E + 1, TB), TB, 0, st>>>(L.key_out, E, N, L.nl_ptr);
  GNN_LAUNCH_CHECK();
  finish_ptr_kernel<<<ceil_div(N + 1, TB), TB, 0, st>>>(L.nl_ptr, N, replace, rowptr);
  GNN_LAUNCH_CHECK();
  if (E > 0) {
    fill_slots_kernel<<<ceil_div(E, TB), TB, 0, st>>>(L.key_out, L.val_out, src, E, N, replace, col,
                                                      csr_eid, L.pos);
    GNN_LAUNCH_CHECK();
  }
  if (replace && N > 0) {
    fill_loops_kernel<<<ceil_div(N, TB), TB, 0, st>>>(rowptr, E, N, col, csr_eid, L.pos);
    GNN_LAUNCH_CHECK();
  }
  // ---- CSC by source ----
  if (E > 0) {
    size_t tb = L.sort_bytes;
    // vals were consumed as input only; rebuild identity (sort does not modify input, but be explicit)
    GNN_HIP_TRY(rocprim::radix_sort_pairs(L.sort_tmp, tb, L.key_src, L.key_out, L.vals, L.val_out,
                                          (size_t)E, 0, bits, st));
  }
  boundaries_kernel<<<ceil_div(E + 1, TB), TB, 0, st>>>(L.key_out, E, N, L.nl_ptr);
  GNN_LAUNCH_CHECK();
  finish_ptr_kernel<<<ceil_div(N + 1, TB), TB, 0, st>>>(L.nl_ptr, N, replace, colptr);
  GNN_LAUNCH_CHECK();
  if (E > 0) {
    fill_slots_kernel<<<ceil_div(E, TB), TB, 0, st>>>(L.key_out, L.val_out, dst, E, N, replace, row,
                                                      L.csc_eid, nullptr);
    GNN_LAUNCH_CHECK();
  }
  if (replace && N > 0) {
    fill_loops_kernel<<<ceil_div(N, TB), TB, 0, st>>>(colptr, E, N, row, L.csc_eid, nullptr);
    GNN_LAUNCH_CHECK();
  }
  csc2csr_kernel<<<ceil_div(Smax > 0 ? Smax : 1, TB), TB, 0, st>>>(colptr, N, Smax, L.csc_eid, L.pos,
                                                                    csc2csr, stats);
  GNN_LAUNCH_CHECK();
  return GNN_OK;
}
