// K0b — long-segment split of a plan direction (CSR rows or CSC columns).
//
// Elliptic-shaped graphs are heavy-tailed: a few hub rows hold hundreds of slots while the
// mean degree is ≈2.3.  A row-per-wave (or row-per-group) gather runs a hub's slots in one
// dependent loop, and that one wave sets the kernel's tail.  The split caps every segment at
// seg_len slots for the main aggregation pass; the rest of a long segment is cut into pieces of
// seg_len slots that separate waves reduce into a small partial-sum buffer, and a combine pass
// adds a long segment's partials in piece order (fixed order: results are reproducible).
//
//   ptr/nbr      the truncated segments (first min(deg, seg_len) slots of each, PyG order kept)
//   order[i]     (optional) degree-ordered main pass: position i of ptr/nbr holds segment
//                order[i]; positions sorted by truncated length, longest first, ties in segment
//                order (stable).  A lane-group gather then gives the groups of one wave segments
//                of (nearly) the same length — no wave waits on one group's long row while the
//                others idle — and the heaviest waves start first.
//   piece0[s]    partial-sum row of piece 0 of a long segment s (pieces of s are consecutive),
//                -1 for a short segment
//   piece_seg[p] the segment of piece p;  long_seg[l] the l-th long segment
// Built once per plan (like the CSR itself); never in the training loop.
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "common.hpp"

namespace gnnmp {
namespace {

__global__ void split_count_kernel(const int32_t* __restrict__ ptr, int64_t n, int32_t T,
                                   unsigned long long* __restrict__ counts) {
  __shared__ unsigned long long red[3][256];
  const int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  unsigned long long tr = 0, lg = 0, pc = 0;
  if (s < n) {
    const int32_t d = ptr[s + 1] - ptr[s];
    tr = (unsigned long long)(d < T ? d : T);
    if (d > T) { lg = 1; pc = (unsigned long long)((d + T - 1) / T); }
  }
  red[0][threadIdx.x] = tr; red[1][threadIdx.x] = lg; red[2][threadIdx.x] = pc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o)
      for (int q = 0; q < 3; ++q) red[q][threadIdx.x] += red[q][threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x < 3) atomicAdd(&counts[threadIdx.x], red[threadIdx.x][0]);  // integer: order-free
}

// Per segment: truncated length, long flag, piece count (inputs of the three scans).
__global__ void split_lens_kernel(const int32_t* __restrict__ ptr, int64_t n, int32_t T,
                                  int32_t* __restrict__ tlen, int32_t* __restrict__ lflag,
                                  int32_t* __restrict__ npc) {
  const int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (s > n) return;
  if (s == n) { tlen[s] = 0; lflag[s] = 0; npc[s] = 0; return; }
  const int32_t d = ptr[s + 1] - ptr[s];
  tlen[s] = d < T ? d : T;
  lflag[s] = d > T ? 1 : 0;
  npc[s] = d > T ? (d + T - 1) / T : 0;
}

__global__ void split_fill_kernel(const int32_t* __restrict__ ptr, const int32_t* __restrict__ nbr, int64_t n,
                                  int32_t T, const int32_t* __restrict__ tptr, const int32_t* __restrict__ lidx,
                                  const int32_t* __restrict__ pscan, int32_t* __restrict__ tnbr,
                                  int32_t* __restrict__ piece0, int32_t* __restrict__ piece_seg,
                                  int32_t* __restrict__ long_seg) {
  const int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (s >= n) return;
  const int32_t b = ptr[s];
  const int32_t d = ptr[s + 1] - b;
  const int32_t L = d < T ? d : T;
  const int32_t o = tptr[s];
  if (tnbr)  // null: the ordered fill writes the truncated slots
    for (int32_t i = 0; i < L; ++i) tnbr[o + i] = nbr[b + i];
  if (d > T) {
    const int32_t p0 = pscan[s];
    piece0[s] = p0;
    long_seg[lidx[s]] = (int32_t)s;
    const int32_t np = (d + T - 1) / T;
    for (int32_t k = 0; k < np; ++k) piece_seg[p0 + k] = (int32_t)s;
  } else {
    piece0[s] = -1;
  }
}

// Degree order: sort key T - tlen (0 for the longest), values the segment ids.
__global__ void split_order_keys_kernel(const int32_t* __restrict__ tlen, int64_t n, int32_t T,
                                        int32_t* __restrict__ key, int32_t* __restrict__ ids) {
  const int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (s >= n) return;
  key[s] = T - tlen[s];
  ids[s] = (int32_t)s;
}

// Truncated length of position i (segment order[i]); position n gets 0 (the scan's total).
__global__ void split_order_lens_kernel(const int32_t* __restrict__ tlen, const int32_t* __restrict__ order,
                                        int64_t n, int32_t* __restrict__ olen) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i > n) return;
  olen[i] = i < n ? tlen[order[i]] : 0;
}

// Ordered fill: position i copies the truncated slots of segment order[i] to tnbr[tptr[i]..];
// the piece tables stay indexed by segment id (pieces in segment order).
__global__ void split_fill_ordered_kernel(const int32_t* __restrict__ ptr, const int32_t* __restrict__ nbr,
                                          int64_t n, int32_t T, const int32_t* __restrict__ order,
                                          const int32_t* __restrict__ tptr, int32_t* __restrict__ tnbr) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t s = order[i];
  const int32_t b = ptr[s];
  const int32_t d = ptr[s + 1] - b;
  const int32_t L = d < T ? d : T;
  const int32_t o = tptr[i];
  for (int32_t k = 0; k < L; ++k) tnbr[o + k] = nbr[b + k];
}

struct SplitLayout {
  int32_t *tlen, *lflag, *npc, *lidx, *pscan;
  int32_t *okey, *okey_out, *oids, *olen, *tmp_ptr;
  void* scan_tmp;
  size_t scan_bytes;
};

gnn_status scan_temp_bytes(int64_t n, size_t* bytes) {
  size_t tb = 0;
  hipError_t e = rocprim::exclusive_scan(nullptr, tb, (const int32_t*)nullptr, (int32_t*)nullptr, 0,
                                         (size_t)(n + 1), rocprim::plus<int32_t>(), (hipStream_t)0);
  if (e != hipSuccess) return hip_check(e, "scan_temp_bytes");
  size_t sb = 0;  // the degree-order sort shares the temporary
  e = rocprim::radix_sort_pairs(nullptr, sb, (int32_t*)nullptr, (int32_t*)nullptr, (int32_t*)nullptr,
                                (int32_t*)nullptr, (size_t)n, 0, 7, (hipStream_t)0);
  if (e != hipSuccess) return hip_check(e, "scan_temp_bytes (sort)");
  *bytes = tb > sb ? tb : sb;
  return GNN_OK;
}

template <typename Carver>
void carve_split(Carver& c, int64_t n, size_t scan_bytes, SplitLayout* L) {
  const size_t m = (size_t)n + 1;
  auto* a = c.template take<int32_t>(m);
  auto* b = c.template take<int32_t>(m);
  auto* d = c.template take<int32_t>(m);
  auto* e = c.template take<int32_t>(m);
  auto* f = c.template take<int32_t>(m);
  auto* k0 = c.template take<int32_t>(m);
  auto* k1 = c.template take<int32_t>(m);
  auto* ids = c.template take<int32_t>(m);
  auto* ol = c.template take<int32_t>(m);
  auto* tp = c.template take<int32_t>(m);
  auto* t = c.template take<char>(scan_bytes);
  if (L) {
    L->tlen = a; L->lflag = b; L->npc = d; L->lidx = e; L->pscan = f;
    L->okey = k0; L->okey_out = k1; L->oids = ids; L->olen = ol; L->tmp_ptr = tp;
    L->scan_tmp = t; L->scan_bytes = scan_bytes;
  }
}

struct SizerAdapter2 {
  WorkspaceSizer s;
  template <typename T>
  T* take(size_t count) { s.take<T>(count); return nullptr; }
};

}  // namespace
}  // namespace gnnmp

using namespace gnnmp;

extern "C" gnn_status gnn_split_workspace_size(int64_t num_segs, size_t* bytes) {
  if (!bytes || num_segs < 0) return fail(GNN_ERR_INVALID_ARG, __func__, "bad args");
  size_t sb = 0;
  gnn_status s = scan_temp_bytes(num_segs, &sb);
  if (s != GNN_OK) return s;
  SizerAdapter2 a;
  carve_split(a, num_segs, sb, nullptr);
  *bytes = a.s.used + 256;
  return GNN_OK;
}

extern "C" gnn_status gnn_split_count(const int32_t* ptr, int64_t num_segs, int32_t seg_len, int64_t* counts,
                                      gnn_stream_t stream) {
  if (!ptr || !counts || num_segs < 0 || seg_len < 1) return fail(GNN_ERR_INVALID_ARG, __func__, "bad args");
  hipStream_t st = (hipStream_t)stream;
  GNN_HIP_TRY(hipMemsetAsync(counts, 0, 3 * sizeof(int64_t), st));
  if (num_segs == 0) return GNN_OK;
  split_count_kernel<<<(unsigned)ceil_div(num_segs, 256), 256, 0, st>>>(
      ptr, num_segs, seg_len, reinterpret_cast<unsigned long long*>(counts));
  GNN_LAUNCH_CHECK();
  return GNN_OK;
}

extern "C" gnn_status gnn_split_build(const int32_t* ptr, const int32_t* nbr, int64_t num_segs, int32_t seg_len,
                                      int32_t* tptr, int32_t* tnbr, int32_t* piece0, int32_t* piece_seg,
                                      int32_t* long_seg, int32_t* order, void* workspace, size_t workspace_bytes,
                                      gnn_stream_t stream) {
  if (!ptr || !tptr || num_segs < 0 || seg_len < 1 || seg_len > 64) return fail(GNN_ERR_INVALID_ARG, __func__, "bad args");
  if (num_segs > 0 && (!piece0 || !tnbr)) return fail(GNN_ERR_INVALID_ARG, __func__, "null output");
  if (num_segs >= INT32_MAX) return fail(GNN_ERR_INVALID_ARG, __func__, "too many segments");
  size_t sb = 0;
  gnn_status s = scan_temp_bytes(num_segs, &sb);
  if (s != GNN_OK) return s;
  WorkspaceCarver c(workspace, workspace_bytes);
  SplitLayout L;
  carve_split(c, num_segs, sb, &L);
  if (!c.ok) return fail(GNN_ERR_WORKSPACE, __func__, "workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const int64_t m = num_segs + 1;
  split_lens_kernel<<<(unsigned)ceil_div(m, 256), 256, 0, st>>>(ptr, num_segs, seg_len, L.tlen, L.lflag, L.npc);
  GNN_LAUNCH_CHECK();
  size_t tb = L.scan_bytes;
  // segment-order pointer of the truncated segments (with an order: scratch for the unordered fill)
  int32_t* sptr = order ? L.tmp_ptr : tptr;
  GNN_HIP_TRY(rocprim::exclusive_scan(L.scan_tmp, tb, L.tlen, sptr, 0, (size_t)m, rocprim::plus<int32_t>(), st));
  tb = L.scan_bytes;
  GNN_HIP_TRY(rocprim::exclusive_scan(L.scan_tmp, tb, L.lflag, L.lidx, 0, (size_t)m, rocprim::plus<int32_t>(), st));
  tb = L.scan_bytes;
  GNN_HIP_TRY(rocprim::exclusive_scan(L.scan_tmp, tb, L.npc, L.pscan, 0, (size_t)m, rocprim::plus<int32_t>(), st));
  if (num_segs > 0) {
    split_fill_kernel<<<(unsigned)ceil_div(num_segs, 256), 256, 0, st>>>(
        ptr, nbr, num_segs, seg_len, sptr, L.lidx, L.pscan, order ? nullptr : tnbr, piece0, piece_seg, long_seg);
    GNN_LAUNCH_CHECK();
  }
  if (order) {  // degree order: stable radix sort of (T - tlen, id), then the ordered pointer and fill
    if (num_segs > 0) {
      split_order_keys_kernel<<<(unsigned)ceil_div(num_segs, 256), 256, 0, st>>>(L.tlen, num_segs, seg_len, L.okey,
                                                                                 L.oids);
      GNN_LAUNCH_CHECK();
      tb = L.scan_bytes;
      GNN_HIP_TRY(rocprim::radix_sort_pairs(L.scan_tmp, tb, L.okey, L.okey_out, L.oids, order, (size_t)num_segs, 0, 7,
                                            st));
    }
    split_order_lens_kernel<<<(unsigned)ceil_div(m, 256), 256, 0, st>>>(L.tlen, order, num_segs, L.olen);
    GNN_LAUNCH_CHECK();
    tb = L.scan_bytes;
    GNN_HIP_TRY(rocprim::exclusive_scan(L.scan_tmp, tb, L.olen, tptr, 0, (size_t)m, rocprim::plus<int32_t>(), st));
    if (num_segs > 0) {
      split_fill_ordered_kernel<<<(unsigned)ceil_div(num_segs, 256), 256, 0, st>>>(ptr, nbr, num_segs, seg_len, order,
                                                                                   tptr, tnbr);
      GNN_LAUNCH_CHECK();
    }
  }
  return GNN_OK;
}
