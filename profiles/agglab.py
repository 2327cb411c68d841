"""Lab build of the aggregation (make -C elliptic_gnn_project_amd/csrc lab): route gnn_aggregate_f32
calls to _lab/libgnnmp_agglab.so, whose gnnx_set_agg_variant selects lab launch shapes.  libgnnmp.so
itself has no runtime knob (the variant is the compile-time constant 0 there)."""
from __future__ import annotations

import ctypes
import os

from elliptic_gnn_project_amd import _lib

LAB_SO = os.path.join(os.path.dirname(_lib.LIB_PATH), "_lab", "libgnnmp_agglab.so")


def route_to_agglab():
    """Load the lab library, send gnn_aggregate_f32 through it; returns gnnx_set_agg_variant."""
    _lib.load()
    if not os.path.exists(LAB_SO):
        raise SystemExit(f"{LAB_SO} missing: make -C elliptic_gnn_project_amd/csrc lab")
    lab = ctypes.CDLL(LAB_SO)
    res, args = _lib.SIGNATURES["gnn_aggregate_f32"]
    lab.gnn_aggregate_f32.restype, lab.gnn_aggregate_f32.argtypes = res, args
    setv = lab.gnnx_set_agg_variant
    setv.argtypes, setv.restype = [ctypes.c_int], None
    prod_call = _lib.call

    def call(name, *a):
        if name == "gnn_aggregate_f32":
            _lib.check(lab.gnn_aggregate_f32(*a), name)
        else:
            prod_call(name, *a)

    _lib.call = call
    return setv
