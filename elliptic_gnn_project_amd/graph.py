"""Graph plans: device CSR/CSC of one ``edge_index``, built once and cached on the tensor.

The reference hands the same ``edge_index`` tensor to every conv call of every epoch
(src/train_gnn.py:320-324 builds it, :387-390 pass it), but eval-time callers pass
modified ones (hub ablation src/train_gnn.py:526-540, robustness.py:65-82).  A plan
is therefore keyed on (tensor identity, in-place version, N, loop mode) and stored
as an attribute of the edge_index tensor itself: it dies with the tensor and is
rebuilt if the tensor is modified in place (``_version`` bump).

HBM layout of a plan (int32 throughout, N+1 / S entries):
    rowptr[N+1], col[S], csr_eid[S]       CSR by target (forward gathers)
    colptr[N+1], row[S], csc2csr[S]       CSC by source (backward gathers)
    deg[N] f32                             slots per target (mean count / GCN degree)
    split (per direction, when a segment has > SPLIT_LEN slots): truncated ptr/nbr laid out
      in degree order with order[N] (position -> segment), piece0[N], piece_seg[pieces],
      long_seg[long]   (K0b, graph_split.hip)
    dinv[N] f32                            GCN deg^-1/2 (REPLACE plans only)
    hub (CSR, graphs of <= K1_HUB_MAX_N nodes): ptr[N+1] / nbr without the slots of the rows with
      deg > K1_HUB_DEG, hubs[H] those rows, ws[W+1] balanced wave starts — K1's hub form
      (gnn_sage_mean_fwd_h2 hub)
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _lib

_ATTR = "_gnnmp_plans"
SPLIT_LEN = 32  # slots per piece of a long segment (K0b)
# K1's hub form (include/gnnmp.h gnn_sage_mean_fwd_h2 hub): K1 runs one wave per 16 rows, so its
# time was set by its heaviest waves — the one holding a degree-~200 hub row, and waves whose 16
# rows happen to be heavy (an average wave walks ~37 slots).  Rows with more than K1_HUB_DEG
# slots go to blocks of their own, and the other rows to waves balanced by slots.  For graphs of
# at most K1_HUB_MAX_N nodes (all, by default; GNNMP_K1_HUB_N overrides, for A/B).
# (32 on large graphs; 16 on graphs of <= 65,536 nodes — a strong-scaling shard, whose gather is
# latency-bound: shorter hub chains, profiles/r66_k1_sweep.txt); GNNMP_K1_HUB_DEG overrides (A/B)
K1_HUB_DEG = int(os.environ.get("GNNMP_K1_HUB_DEG", "0"))
# rows per balanced wave on average: 8 on large graphs (the full headline graph: 0.2986 vs 0.3025
# ms/step at 16, four interleaved repetitions, profiles/r58_k1_rows.txt), 4 on graphs of <= 32,768
# nodes (the 8-way shard's gather 17.9 -> 14.1 us with hub degree 16, once the riding B prep no
# longer set K1's length: r66_k1_sweep.txt); GNNMP_K1_WAVE_ROWS overrides (A/B)
K1_WAVE_ROWS = int(os.environ.get("GNNMP_K1_WAVE_ROWS", "0"))
K1_HUB_MAX_N = int(os.environ.get("GNNMP_K1_HUB_N", str(1 << 62)))


def _split_enabled() -> bool:
    return os.environ.get("GNNMP_SPLIT", "1") != "0"


def _order_enabled() -> bool:
    """Degree-ordered main pass of split directions (GNNMP_ORDER=0: plan order, for A/B timing)."""
    return os.environ.get("GNNMP_ORDER", "1") != "0"


def _build_split(lib, ptr: torch.Tensor, nbr: torch.Tensor, n: int, T: int, dev):
    """Long-segment split of one direction; None when no segment exceeds T slots."""
    counts = torch.zeros(3, dtype=torch.int64, device=dev)
    with torch.cuda.device(dev):
        stream = _lib.stream_handle(dev)
        _lib.check(lib.gnn_split_count(ptr.data_ptr(), n, T, counts.data_ptr(), stream), "gnn_split_count")
        s_trunc, n_long, n_pieces = (int(v) for v in counts.cpu())  # one sync per plan build
        if n_long == 0:
            return None
        i32 = dict(dtype=torch.int32, device=dev)
        t = {
            "ptr": torch.empty(n + 1, **i32),
            "nbr": torch.empty(max(s_trunc, 1), **i32),
            "piece0": torch.empty(max(n, 1), **i32),
            "piece_seg": torch.empty(max(n_pieces, 1), **i32),
            "long_seg": torch.empty(max(n_long, 1), **i32),
            "order": torch.empty(max(n, 1), **i32) if _order_enabled() else None,
        }
        nb = _lib.c_size(0)
        _lib.check(lib.gnn_split_workspace_size(n, nb), "gnn_split_workspace_size")
        ws = torch.empty(max(int(nb.value), 1), dtype=torch.uint8, device=dev)
        _lib.check(lib.gnn_split_build(ptr.data_ptr(), nbr.data_ptr(), n, T, t["ptr"].data_ptr(),
                                       t["nbr"].data_ptr(), t["piece0"].data_ptr(), t["piece_seg"].data_ptr(),
                                       t["long_seg"].data_ptr(), _lib.ptr(t["order"]), ws.data_ptr(), ws.numel(),
                                       stream),
                   "gnn_split_build")
        torch.cuda.current_stream(dev).synchronize()  # ws is freed below
    t["c"] = _lib.GnnSplit(T, 0, n_long, n_pieces, t["ptr"].data_ptr(), t["nbr"].data_ptr(),
                           t["piece0"].data_ptr(), t["piece_seg"].data_ptr(), t["long_seg"].data_ptr(),
                           _lib.ptr(t["order"]))
    return t


def _wave_starts(slots: torch.Tensor, n: int) -> torch.Tensor:
    """Row boundaries of K1's balanced main-pass waves: as many waves as 8 (large graphs) or 16
    rows each would take,
    contiguous row ranges of about equal cost (slots + kappa per row: a row's flush costs about a
    slot, and kappa >= mean degree / 2 keeps a wave under 63 rows), doubled until no wave holds
    more than 63 rows (the kernel keeps one row pointer per lane)."""
    kappa = max(1.0, float(slots.sum()) / max(n, 1) / 2.0)
    cost = slots.to(torch.float64) + kappa
    before = torch.cumsum(cost, 0) - cost  # cost of the rows before each row
    rows = K1_WAVE_ROWS if K1_WAVE_ROWS > 0 else (4 if n <= 32768 else 8)
    waves = max(1, -(-n // rows))
    while True:
        target = float(cost.sum()) / waves
        k = torch.arange(waves + 1, dtype=torch.float64, device=slots.device) * target
        b = torch.searchsorted(before, k).clamp_(max=n)
        b[0], b[-1] = 0, n
        if int((b[1:] - b[:-1]).max()) <= 63 or waves >= n:
            return b.to(torch.int32)
        waves = min(2 * waves, n)


def _build_hub(rowptr: torch.Tensor, col: torch.Tensor, deg: torch.Tensor, n: int, T: int):
    """K1's hub form of the CSR: the rows with deg > T (deg: the plan's f32 slot counts, the array
    K1 divides by), the CSR without their slots, in natural order, and the balanced main-pass
    waves over what is left (include/gnnmp.h gnn_sage_mean_fwd_h2 hub)."""
    hub = deg[:n] > T
    nh = int(hub.sum())  # one sync per plan build
    cnt = (rowptr[1:] - rowptr[:-1]).to(torch.int64)
    left = torch.where(hub, 0, cnt)
    t = {"ws": _wave_starts(left, n)}
    if nh:
        ptr = torch.zeros(n + 1, dtype=torch.int64, device=rowptr.device)
        torch.cumsum(left, 0, out=ptr[1:])
        keep = torch.repeat_interleave(~hub, cnt)
        t.update(ptr=ptr.to(torch.int32), nbr=col[: keep.numel()][keep].contiguous(),
                 hubs=torch.nonzero(hub).flatten().to(torch.int32))
        if t["nbr"].numel() == 0:
            t["nbr"] = torch.zeros(1, dtype=torch.int32, device=rowptr.device)
    t["c"] = _lib.GnnSplit(T, 0, nh, t["ws"].numel() - 1, _lib.ptr(t.get("ptr")), _lib.ptr(t.get("nbr")), None,
                           t["ws"].data_ptr(), _lib.ptr(t.get("hubs")), None)
    return t


class GraphPlan:
    """Stable CSR (by target) + CSC (by source) of ``edge_index`` on the HIP device."""

    def __init__(self, edge_index: torch.Tensor, num_nodes: int, loops: int):
        if edge_index.dim() != 2 or edge_index.size(0) != 2:
            raise ValueError(f"edge_index must be [2, E], got {tuple(edge_index.shape)}")
        if edge_index.device.type != "cuda":
            raise RuntimeError(
                "elliptic_gnn_project_amd runs on the MI355X (HIP) device only; "
                f"edge_index is on {edge_index.device}"
            )
        dev = edge_index.device
        N = int(num_nodes)
        E = int(edge_index.size(1))
        self.num_nodes = N
        self.num_edges = E
        self.loops = loops
        self.device = dev
        ei = edge_index.to(torch.int64).contiguous()
        smax = E + (N if loops == _lib.LOOPS_REPLACE else 0)
        i32 = dict(dtype=torch.int32, device=dev)
        self.rowptr = torch.empty(N + 1, **i32)
        self.colptr = torch.empty(N + 1, **i32)
        self.col = torch.empty(max(smax, 1), **i32)
        self.csr_eid = torch.empty(max(smax, 1), **i32)
        self.row = torch.empty(max(smax, 1), **i32)
        self.csc2csr = torch.empty(max(smax, 1), **i32)
        stats = torch.zeros(4, **i32)
        lib = _lib.load()
        ws_bytes = _lib.c_size(0)
        _lib.check(lib.gnn_graph_workspace_size(N, E, ws_bytes), "gnn_graph_workspace_size")
        ws = torch.empty(max(int(ws_bytes.value), 1), dtype=torch.uint8, device=dev)
        with torch.cuda.device(dev):
            stream = _lib.stream_handle(dev)
            _lib.check(
                lib.gnn_graph_build(
                    ei.data_ptr(), E, N, loops,
                    self.rowptr.data_ptr(), self.col.data_ptr(), self.csr_eid.data_ptr(),
                    self.colptr.data_ptr(), self.row.data_ptr(), self.csc2csr.data_ptr(),
                    stats.data_ptr(), ws.data_ptr(), ws.numel(), stream,
                ),
                "gnn_graph_build",
            )
            st = stats.cpu()  # one host sync per plan build (never in the training loop)
        del ws
        if int(st[2]) > 0:
            raise IndexError(
                f"edge_index holds {int(st[2])} entries outside [0, {N}) "
                "(PyG would raise in index_select)"
            )
        self.num_slots = int(st[0])
        self.num_input_loops = int(st[1])
        self.c_graph = _lib.GnnGraph(
            N, self.num_slots,
            self.rowptr.data_ptr(), self.col.data_ptr(),
            self.colptr.data_ptr(), self.row.data_ptr(), self.csc2csr.data_ptr(),
        )
        # long-segment splits of both directions (K0b): hubs no longer set the gather's tail
        self.split_len = SPLIT_LEN if _split_enabled() else 0
        self._splits = {}
        if self.split_len > 0 and self.num_slots > 0:
            for name, ptr, nbr in (("csr", self.rowptr, self.col), ("csc", self.colptr, self.row)):
                sp = _build_split(lib, ptr, nbr, N, self.split_len, dev)
                if sp is not None:
                    self._splits[name] = sp
                    setattr(self.c_graph, f"{name}_split", ctypes.pointer(sp["c"]))
        self.deg = torch.empty(max(N, 1), dtype=torch.float32, device=dev)
        with torch.cuda.device(dev):
            _lib.check(lib.gnn_in_degree_f32(self.c_graph, self.deg.data_ptr(), _lib.stream_handle(dev)),
                       "gnn_in_degree_f32")
        self._dinv = None
        self._hub = False  # built on first use (only the half-pair K1 reads it)

    @property
    def hub(self):
        """K1's hub form (include/gnnmp.h gnn_sage_mean_fwd_h2 hub), or None.  Built lazily, on the
        first half-pair mean over this plan: GCN / GAT / REPLACE plans and the NeighborLoader's
        per-batch plans never pay its host syncs and CSR copy.  Not buildable while a
        stream is being captured — the warm-up forward that precedes every capture builds it."""
        if self._hub is False:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("GraphPlan.hub is built by the first half-pair mean over the plan (host "
                                   "syncs): run one eager forward before capturing the step")
            N = self.num_nodes
            T = K1_HUB_DEG if K1_HUB_DEG > 0 else (16 if N <= 65536 else 32)
            self._hub = (_build_hub(self.rowptr, self.col, self.deg, N, T)
                         if 0 < N <= K1_HUB_MAX_N else None)
        return self._hub

    @property
    def dinv(self) -> torch.Tensor:
        """GCN normalisation deg^-1/2 (PyG gcn_norm); only meaningful on REPLACE plans."""
        if self._dinv is None:
            if self.loops != _lib.LOOPS_REPLACE:
                raise RuntimeError("gcn norm needs a self-loop-replaced plan")
            d = torch.empty(max(self.num_nodes, 1), dtype=torch.float32, device=self.device)
            with torch.cuda.device(self.device):
                _lib.call("gnn_gcn_norm_f32", self.c_graph, d.data_ptr(), _lib.stream_handle(self.device))
            self._dinv = d
        return self._dinv

    def split_pieces(self, transpose: bool) -> int:
        """Partial-sum rows an aggregation over this direction needs (0: unsplit)."""
        sp = self._splits.get("csc" if transpose else "csr")
        return int(sp["c"].num_pieces) if sp is not None else 0

    def csr(self):
        """(rowptr, col, csr_eid) trimmed to the used slots — for tests / inspection."""
        S = self.num_slots
        return self.rowptr, self.col[:S], self.csr_eid[:S]

    def csc(self):
        S = self.num_slots
        return self.colptr, self.row[:S], self.csc2csr[:S]


def get_plan(edge_index: torch.Tensor, num_nodes: int, loops: int = _lib.LOOPS_KEEP) -> GraphPlan:
    """Cached plan for (edge_index, N, loop mode); rebuilt when edge_index changes in place."""
    key = (int(num_nodes), int(loops))
    version = edge_index._version
    plans = getattr(edge_index, _ATTR, None)
    if plans is None or plans.get("version") != version or plans.get("ptr") != edge_index.data_ptr():
        plans = {"version": version, "ptr": edge_index.data_ptr()}
        try:
            setattr(edge_index, _ATTR, plans)
        except (AttributeError, RuntimeError):  # e.g. inference tensors: no caching
            pass
    plan = plans.get(key)
    if plan is None:
        plan = GraphPlan(edge_index, num_nodes, loops)
        plans[key] = plan
    return plan
