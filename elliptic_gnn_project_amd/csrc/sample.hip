// K11 — NeighborLoader neighbour sampling (the mini-batch path of src/train_gnn.py:212-245,329-348).
//
// The reference builds `NeighborLoader(data, num_neighbors=fanout, batch_size, input_nodes,
// shuffle)` (torch_geometric 2.5.3 + pyg-lib `neighbor_sample`, CSC of the in-edges) and trains
// on `logits[:batch.batch_size]`.  Per batch of distinct seed nodes this file samples, hop by
// hop, up to fanout[h] in-neighbours of every node discovered in the previous hop (the seeds for
// hop 0) WITHOUT replacement, de-duplicates the sampled nodes against everything already in the
// batch (disjoint = False), and emits the relabelled subgraph:
//   n_id[0, B)            = the seeds, in order;  then each hop's new nodes in order of their
//                           first appearance in that hop's edge list
//   (e_src, e_dst)[s]     = (local neighbour, local frontier node): messages flow e_src -> e_dst,
//                           the direction of the original edge; e_id[s] = its PyG edge id
//   edge order            = hop, then frontier node, then CSR (= PyG edge) order of the picks.
// Randomness is a counter hash of (seed, hop, node, draw), so a batch is a pure function of
// (graph, seeds, fanout, seed): reproducible, and independent of launch geometry.  PyG's own
// draws come from its RNG stream and cannot be matched; the tests check the sampler's contract
// (fan-out bounds, edges ⊆ graph, dedup/relabel, hop structure, determinism) instead.
//
// HBM work is small next to a training step (one pass over the frontier's CSR rows per hop);
// every pass is one thread per frontier node or per sampled edge.  Output sizes are data
// dependent, so each hop reads two counts back to the host (the only host syncs).
#include <climits>
#include <type_traits>
#include <rocprim/device/device_scan.hpp>

#include "common.hpp"

namespace gnnmp {
namespace {

constexpr int kMaxFanout = 256;  // per-thread Floyd sample buffer (scratch)

__device__ __forceinline__ uint32_t sample_hash(uint64_t seed, uint32_t hop, uint32_t node, uint32_t draw) {
  uint64_t z = seed ^ (0x9E3779B97F4A7C15ull * (((uint64_t)hop << 32) | node)) ^ ((uint64_t)draw * 0xD1B54A32D192ED03ull);
  z ^= z >> 30;
  z *= 0xBF58476D1CE4E5B9ull;
  z ^= z >> 27;
  z *= 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)(z >> 32);
}

__global__ void sample_init_kernel(int32_t* __restrict__ nodemap, int32_t* __restrict__ first, int64_t N) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= N) return;
  nodemap[i] = -1;
  first[i] = INT_MAX;
}

// seeds -> local ids 0..B-1; flags[0] counts out-of-range seeds, flags[1] duplicates
__global__ void sample_seed_kernel(const int32_t* __restrict__ seeds, int64_t B, int64_t N, int32_t* __restrict__ nodemap,
                                   int32_t* __restrict__ n_id, int32_t* __restrict__ flags) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= B) return;
  const int32_t v = seeds[i];
  if (v < 0 || v >= N) {
    atomicAdd(&flags[0], 1);
    n_id[i] = 0;
    return;
  }
  if (atomicCAS(&nodemap[v], -1, (int32_t)i) != -1) atomicAdd(&flags[1], 1);
  n_id[i] = v;
}

// cnt[i] = picks of frontier node i (min(in-degree, fanout); fanout < 0: all); cnt[n] = 0
__global__ void sample_count_kernel(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ frontier, int64_t n,
                                    int32_t fanout, int32_t* __restrict__ cnt) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i > n) return;
  if (i == n) {
    cnt[i] = 0;
    return;
  }
  const int32_t v = frontier[i];
  const int32_t d = rowptr[v + 1] - rowptr[v];
  cnt[i] = fanout < 0 ? d : min(d, fanout);
}

// One thread per frontier node: all in-neighbours when deg <= fanout, else a uniform
// fanout-subset of the CSR positions (Floyd's algorithm), emitted in ascending position order.
__global__ void sample_fill_kernel(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                                   const int32_t* __restrict__ csr_eid, const int32_t* __restrict__ frontier, int64_t n,
                                   int32_t base, const int32_t* __restrict__ cnt, const int32_t* __restrict__ off,
                                   uint64_t seed, uint32_t hop, int32_t* __restrict__ e_src, int32_t* __restrict__ e_dst,
                                   int32_t* __restrict__ e_id) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t v = frontier[i];
  const int32_t r0 = rowptr[v], d = rowptr[v + 1] - r0, c = cnt[i], o = off[i];
  const int32_t me = base + (int32_t)i;
  auto emit = [&](int j, int32_t pos) {
    const int32_t p = r0 + pos;
    e_src[o + j] = col[p];  // global id; relabelled after the dedup
    e_dst[o + j] = me;
    e_id[o + j] = csr_eid ? csr_eid[p] : p;
  };
  if (c == d) {
    for (int j = 0; j < d; ++j) emit(j, j);
    return;
  }
  if (c > kMaxFanout) {  // more picks than the Floyd buffer: selection sampling (Knuth's
    // algorithm S) — slot j kept with probability need / (d - j), one pass, already in CSR order
    int32_t need = c, m = 0;
    for (int32_t j = 0; j < d && need > 0; ++j) {
      const uint64_t u = sample_hash(seed, hop, (uint32_t)v, (uint32_t)j);
      if (((u * (uint64_t)(d - j)) >> 32) < (uint64_t)need) {
        emit(m++, j);
        --need;
      }
    }
    return;
  }
  int32_t sel[kMaxFanout];
  int m = 0;
  for (int32_t j = d - c; j < d; ++j) {
    const int32_t t = (int32_t)(((uint64_t)sample_hash(seed, hop, (uint32_t)v, (uint32_t)j) * (uint64_t)(j + 1)) >> 32);
    bool dup = false;
    for (int q = 0; q < m; ++q) dup |= sel[q] == t;
    sel[m++] = dup ? j : t;
  }
  for (int a = 1; a < m; ++a) {  // insertion sort: picks in CSR order
    const int32_t x = sel[a];
    int b = a - 1;
    while (b >= 0 && sel[b] > x) {
      sel[b + 1] = sel[b];
      --b;
    }
    sel[b + 1] = x;
  }
  for (int j = 0; j < m; ++j) emit(j, sel[j]);
}

// first appearance of every not-yet-mapped neighbour in this hop's edge list
__global__ void sample_mark_kernel(const int32_t* __restrict__ e_src, int64_t E, const int32_t* __restrict__ nodemap,
                                   int32_t* __restrict__ first) {
  const int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (s >= E) return;
  const int32_t u = e_src[s];
  if (nodemap[u] < 0) atomicMin(&first[u], (int32_t)s);
}

__global__ void sample_flag_kernel(const int32_t* __restrict__ e_src, int64_t E, const int32_t* __restrict__ nodemap,
                                   const int32_t* __restrict__ first, int32_t* __restrict__ flag) {
  const int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (s > E) return;
  if (s == E) {
    flag[s] = 0;
    return;
  }
  const int32_t u = e_src[s];
  flag[s] = (nodemap[u] < 0 && first[u] == (int32_t)s) ? 1 : 0;
}

__global__ void sample_assign_kernel(const int32_t* __restrict__ e_src, int64_t E, const int32_t* __restrict__ flag,
                                     const int32_t* __restrict__ rank, int32_t n0, int32_t* __restrict__ nodemap,
                                     int32_t* __restrict__ n_id) {
  const int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (s >= E || !flag[s]) return;
  const int32_t u = e_src[s], id = n0 + rank[s];
  nodemap[u] = id;
  n_id[id] = u;
}

__global__ void sample_relabel_kernel(int32_t* __restrict__ e_src, int64_t E, const int32_t* __restrict__ nodemap) {
  const int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (s >= E) return;
  e_src[s] = nodemap[e_src[s]];
}

inline unsigned blocks(int64_t n) { return (unsigned)std::max<int64_t>(1, ceil_div(n, 256)); }

size_t scan_temp_bytes(int64_t n) {
  size_t b = 0;
  (void)rocprim::exclusive_scan(nullptr, b, (const int32_t*)nullptr, (int32_t*)nullptr, 0, (size_t)n, rocprim::plus<int32_t>(),
                          (hipStream_t)0);
  return b;
}

struct SampleLayout {
  int32_t *nodemap, *first, *cnt, *off, *flag, *rank, *dev_counts;
  void* scan_tmp;
  size_t scan_bytes;
};

template <typename C>
void carve_sample(C& c, int64_t N, int64_t node_cap, int64_t edge_cap, SampleLayout* L) {
  const size_t sb = std::max<size_t>(scan_temp_bytes(node_cap + 1), scan_temp_bytes(edge_cap + 1));
  if constexpr (std::is_same_v<C, WorkspaceCarver>) {
    L->nodemap = c.template take<int32_t>(N);
    L->first = c.template take<int32_t>(N);
    L->cnt = c.template take<int32_t>(node_cap + 1);
    L->off = c.template take<int32_t>(node_cap + 1);
    L->flag = c.template take<int32_t>(edge_cap + 1);
    L->rank = c.template take<int32_t>(edge_cap + 1);
    L->dev_counts = c.template take<int32_t>(4);
    L->scan_tmp = c.template take<char>(sb);
    L->scan_bytes = sb;
  } else {
    c.template take<int32_t>(N);
    c.template take<int32_t>(N);
    c.template take<int32_t>(node_cap + 1);
    c.template take<int32_t>(node_cap + 1);
    c.template take<int32_t>(edge_cap + 1);
    c.template take<int32_t>(edge_cap + 1);
    c.template take<int32_t>(4);
    c.template take<char>(sb);
  }
}

}  // namespace
}  // namespace gnnmp

using namespace gnnmp;

extern "C" gnn_status gnn_neighbor_sample_workspace_size(int64_t num_nodes, int64_t node_cap, int64_t edge_cap,
                                                         size_t* bytes) {
  if (!bytes || num_nodes < 0 || node_cap < 0 || edge_cap < 0)
    return fail(GNN_ERR_INVALID_ARG, __func__, "bad sizes");
  WorkspaceSizer s;
  SampleLayout L{};
  carve_sample(s, std::max<int64_t>(num_nodes, 1), node_cap, edge_cap, &L);
  *bytes = s.used;
  return GNN_OK;
}

extern "C" gnn_status gnn_neighbor_sample(const gnn_graph* g, const int32_t* csr_eid, const int32_t* seeds,
                                          int64_t num_seeds, int32_t num_hops, const int32_t* fanout, uint64_t seed,
                                          int32_t* n_id, int64_t node_cap, int32_t* e_src, int32_t* e_dst,
                                          int32_t* e_id, int64_t edge_cap, int64_t* hop_nodes, int64_t* hop_edges,
                                          void* workspace, size_t workspace_bytes, gnn_stream_t stream) {
  const char* fn = __func__;
  if (!g || !g->rowptr || (!g->col && g->num_slots > 0)) return fail(GNN_ERR_INVALID_ARG, fn, "graph plan required");
  if (num_seeds < 0 || num_hops < 0 || (num_hops > 0 && !fanout) || !hop_nodes || !hop_edges)
    return fail(GNN_ERR_INVALID_ARG, fn, "bad arguments");
  if (num_seeds > node_cap || (num_seeds > 0 && (!seeds || !n_id)))
    return fail(GNN_ERR_INVALID_ARG, fn, "node_cap smaller than the seed count");
  for (int h = 0; h < num_hops; ++h)
    if (fanout[h] == 0 || fanout[h] < -1)
      return fail(GNN_ERR_INVALID_ARG, fn, "fanout must be -1 (all) or >= 1");
  const int64_t N = g->num_nodes;
  if (N >= INT_MAX || node_cap >= INT_MAX || edge_cap >= INT_MAX) return fail(GNN_ERR_INVALID_ARG, fn, "int32 sizes");
  WorkspaceCarver c(workspace, workspace_bytes);
  SampleLayout L{};
  carve_sample(c, std::max<int64_t>(N, 1), node_cap, edge_cap, &L);
  if (!c.ok) return fail(GNN_ERR_INVALID_ARG, fn, "workspace too small");
  hipStream_t st = static_cast<hipStream_t>(stream);
  for (int h = 0; h <= num_hops; ++h) hop_nodes[h] = 0;
  for (int h = 0; h < num_hops; ++h) hop_edges[h] = 0;
  if (num_seeds == 0) return GNN_OK;

  sample_init_kernel<<<blocks(N), 256, 0, st>>>(L.nodemap, L.first, N);
  GNN_HIP_TRY(hipMemsetAsync(L.dev_counts, 0, 4 * sizeof(int32_t), st));
  sample_seed_kernel<<<blocks(num_seeds), 256, 0, st>>>(seeds, num_seeds, N, L.nodemap, n_id, L.dev_counts);
  GNN_LAUNCH_CHECK();
  int32_t hc[4];
  GNN_HIP_TRY(hipMemcpyAsync(hc, L.dev_counts, sizeof(hc), hipMemcpyDeviceToHost, st));
  GNN_HIP_TRY(hipStreamSynchronize(st));
  if (hc[0]) return fail(GNN_ERR_INDEX_OUT_OF_RANGE, fn, "seed node outside [0, num_nodes)");
  if (hc[1]) return fail(GNN_ERR_INVALID_ARG, fn, "seed nodes must be distinct");

  int64_t nn = num_seeds, ne = 0, fbeg = 0, fend = num_seeds;
  hop_nodes[0] = num_seeds;
  for (int h = 0; h < num_hops; ++h) {
    const int64_t nf = fend - fbeg;
    if (nf == 0) {
      hop_nodes[h + 1] = 0;
      continue;
    }
    const int32_t* frontier = n_id + fbeg;
    sample_count_kernel<<<blocks(nf + 1), 256, 0, st>>>(g->rowptr, frontier, nf, fanout[h], L.cnt);
    GNN_HIP_TRY(rocprim::exclusive_scan(L.scan_tmp, L.scan_bytes, L.cnt, L.off, 0, (size_t)(nf + 1),
                                        rocprim::plus<int32_t>(), st));
    int32_t eh = 0;
    GNN_HIP_TRY(hipMemcpyAsync(&eh, L.off + nf, sizeof(int32_t), hipMemcpyDeviceToHost, st));
    GNN_HIP_TRY(hipStreamSynchronize(st));
    if (ne + eh > edge_cap) return fail(GNN_ERR_INVALID_ARG, fn, "edge_cap too small for the sampled edges");
    int32_t* es = e_src + ne;
    sample_fill_kernel<<<blocks(nf), 256, 0, st>>>(g->rowptr, g->col, csr_eid, frontier, nf, (int32_t)fbeg, L.cnt,
                                                   L.off, seed, (uint32_t)h, es, e_dst + ne, e_id + ne);
    GNN_LAUNCH_CHECK();
    sample_mark_kernel<<<blocks(eh), 256, 0, st>>>(es, eh, L.nodemap, L.first);
    sample_flag_kernel<<<blocks(eh + 1), 256, 0, st>>>(es, eh, L.nodemap, L.first, L.flag);
    GNN_HIP_TRY(rocprim::exclusive_scan(L.scan_tmp, L.scan_bytes, L.flag, L.rank, 0, (size_t)(eh + 1),
                                        rocprim::plus<int32_t>(), st));
    int32_t nnew = 0;
    GNN_HIP_TRY(hipMemcpyAsync(&nnew, L.rank + eh, sizeof(int32_t), hipMemcpyDeviceToHost, st));
    GNN_HIP_TRY(hipStreamSynchronize(st));
    if (nn + nnew > node_cap) return fail(GNN_ERR_INVALID_ARG, fn, "node_cap too small for the sampled nodes");
    sample_assign_kernel<<<blocks(eh), 256, 0, st>>>(es, eh, L.flag, L.rank, (int32_t)nn, L.nodemap, n_id);
    sample_relabel_kernel<<<blocks(eh), 256, 0, st>>>(es, eh, L.nodemap);
    GNN_LAUNCH_CHECK();
    hop_edges[h] = eh;
    hop_nodes[h + 1] = nnew;
    fbeg = nn;
    nn += nnew;
    fend = nn;
    ne += eh;
  }
  return GNN_OK;
}
