"""GPU: the degree-ordered main pass of split plan directions (K0b ``order``, graph_split.hip).

* the tables are bit-exact against numpy: ``order`` = a stable sort of the segments by truncated
  length, longest first; the ordered truncated pointer / neighbour arrays are the plan-order ones
  permuted by it; the piece tables are unchanged (segment-indexed);
* every aggregation mode that takes the split (8 < F <= 128: the lane-group gather) gives results
  BITWISE equal to the plan-order pass: the order changes which lane group sums a row, never the
  sequence a row is summed in (aggregate.hip also builds without FMA contraction, so a walk's
  shape cannot change a rounding).
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _plans(ei, n, loops, device):
    from elliptic_gnn_project_amd.graph import get_plan

    out = {}
    old = os.environ.get("GNNMP_ORDER")
    try:
        for o in ("0", "1"):
            os.environ["GNNMP_ORDER"] = o
            out[o] = get_plan(ei.clone().to(device), n, loops)
    finally:
        if old is None:
            os.environ.pop("GNNMP_ORDER", None)
        else:
            os.environ["GNNMP_ORDER"] = old
    return out


def _graph(sym, n=30000, e=40000, seed=5):
    from elliptic_gnn_project_amd.dataset_elliptic import prepare_inputs, synthetic_elliptic

    return prepare_inputs(synthetic_elliptic(num_nodes=n, num_edges=e, seed=seed),
                          dict(use_time_scalar=True, symmetrize_edges=sym, train_window_k=10))


@pytest.mark.parametrize("loops_name", ["keep", "replace"])
def test_order_tables_bit_exact(device, loops_name):
    from elliptic_gnn_project_amd import _lib

    loops = _lib.LOOPS_KEEP if loops_name == "keep" else _lib.LOOPS_REPLACE
    g = _graph(loops_name == "keep")
    pl = _plans(g.edge_index, g.x.size(0), loops, device)
    assert pl["1"]._splits, "the test graph must have long segments"
    for name in pl["1"]._splits:
        a, b = pl["0"]._splits[name], pl["1"]._splits[name]
        assert a["order"] is None and b["order"] is not None
        T = pl["1"].split_len
        tptr = a["ptr"].cpu().numpy().astype(np.int64)
        tnbr = a["nbr"].cpu().numpy()
        tlen = np.diff(tptr)
        order = np.argsort(T - tlen, kind="stable")
        np.testing.assert_array_equal(b["order"].cpu().numpy(), order)
        optr = np.concatenate([[0], np.cumsum(tlen[order])])
        np.testing.assert_array_equal(b["ptr"].cpu().numpy(), optr)
        onbr = np.concatenate([tnbr[tptr[s]: tptr[s + 1]] for s in order]) if order.size else tnbr[:0]
        np.testing.assert_array_equal(b["nbr"][: onbr.size].cpu().numpy(), onbr)
        for k in ("piece0", "piece_seg", "long_seg"):
            assert torch.equal(a[k], b[k]), k


CASES = [  # (graph symmetrized, loops, mode name, transpose, F, epilogue)
    (True, "keep", "MEAN", False, 64, {}),
    (True, "keep", "MEAN_BWD", True, 64, {}),
    (True, "keep", "MEAN", False, 128, dict(relu=True)),
    (True, "keep", "SUM", False, 16, {}),
    (False, "replace", "GCN", False, 64, dict(relu=True, dropout_p=0.5, seed=7)),
    (False, "replace", "GCN", True, 64, {}),
    (True, "keep", "MEAN", False, 64, dict(addend=True, relu=True)),
]


@pytest.mark.parametrize("sym,loops_name,mode,transpose,F,epi", CASES)
def test_ordered_pass_bitwise_equals_plan_order(device, sym, loops_name, mode, transpose, F, epi):
    from elliptic_gnn_project_amd import _lib
    from elliptic_gnn_project_amd.aggregation import aggregate

    loops = _lib.LOOPS_KEEP if loops_name == "keep" else _lib.LOOPS_REPLACE
    g = _graph(sym)
    N = g.x.size(0)
    pl = _plans(g.edge_index, N, loops, device)
    gen = torch.Generator().manual_seed(F)
    x = torch.randn(N, F, generator=gen).to(device)
    kw = dict(epi)
    if kw.pop("addend", False):
        kw["addend"] = torch.randn(N, F, generator=gen).to(device)
    kw["bias"] = torch.randn(F, generator=gen).to(device)
    outs = []
    for o in ("0", "1"):
        p = pl[o]
        nodew = p.dinv if mode == "GCN" else p.deg
        outs.append(aggregate(p, x, getattr(_lib, f"AGG_{mode}"), transpose=transpose, nodew=nodew, **kw))
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("sym,loops_name,mode,transpose,F,epi", [c for c in CASES if c[4] == 64])
def test_pieces_in_main_launch_bitwise(device, monkeypatch, sym, loops_name, mode, transpose, F, epi):
    """16-lane groups (F = 64): the split pieces walked inside the main pass's launch
    (agg_flat_pieces_kernel) give the results of the separate piece launch bit for bit.  The
    separate-launch shape is selected on the LAB build of aggregate.hip (`make lab`:
    _lab/libgnnmp_agglab.so, gnnx_set_agg_variant(16)); libgnnmp.so has no runtime knob, and its
    own result (the product path) must equal both."""
    import ctypes
    import os

    from elliptic_gnn_project_amd import _lib
    from elliptic_gnn_project_amd.aggregation import aggregate

    lab_so = os.path.join(os.path.dirname(_lib.LIB_PATH), "_lab", "libgnnmp_agglab.so")
    if not os.path.exists(lab_so):
        pytest.skip("lab build missing (make -C elliptic_gnn_project_amd/csrc lab)")
    loops = _lib.LOOPS_KEEP if loops_name == "keep" else _lib.LOOPS_REPLACE
    g = _graph(sym)
    N = g.x.size(0)
    p = _plans(g.edge_index, N, loops, device)["1"]
    if p.split_pieces(transpose) == 0:
        pytest.skip("no long segments in this direction (the directed graph's out-degrees)")
    gen = torch.Generator().manual_seed(F + 1)
    x = torch.randn(N, F, generator=gen).to(device)
    kw = dict(epi)
    if kw.pop("addend", False):
        kw["addend"] = torch.randn(N, F, generator=gen).to(device)
    kw["bias"] = torch.randn(F, generator=gen).to(device)
    nodew = p.dinv if mode == "GCN" else p.deg
    agg_mode = getattr(_lib, f"AGG_{mode}")
    prod = aggregate(p, x, agg_mode, transpose=transpose, nodew=nodew, **kw)
    lab = ctypes.CDLL(lab_so)
    res, args = _lib.SIGNATURES["gnn_aggregate_f32"]
    lab.gnn_aggregate_f32.restype, lab.gnn_aggregate_f32.argtypes = res, args
    lab.gnnx_set_agg_variant.argtypes, lab.gnnx_set_agg_variant.restype = [ctypes.c_int], None
    prod_call = _lib.call
    monkeypatch.setattr(_lib, "call", lambda name, *a: _lib.check(lab.gnn_aggregate_f32(*a), name)
                        if name == "gnn_aggregate_f32" else prod_call(name, *a))
    outs = []
    for v in (0, 16):
        lab.gnnx_set_agg_variant(v)
        outs.append(aggregate(p, x, agg_mode, transpose=transpose, nodew=nodew, **kw))
    lab.gnnx_set_agg_variant(0)
    assert torch.equal(prod, outs[0])
    assert torch.equal(outs[0], outs[1])
