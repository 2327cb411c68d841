"""ORACLE (test infrastructure only) — bit-exact mirror of libgnnmp's dropout mask.

libgnnmp's fused epilogue (csrc/gemm_f32.hip: keep_elem) keeps element ``idx = row*cols + col``
of a call seeded with ``seed`` iff  top24(splitmix64(seed ^ idx*0xD1B54A32D192ED03)) <
(uint32)((1 - (double)p) * 2^24), where p is the float32 dropout probability, and scales kept
values by 1/(1-p) — the semantics of F.dropout (src/models/gnn.py:30,51), with a counter hash
in place of torch's Philox stream.  The CPU oracle applies this exact mask so train-mode
steps can be compared element for element.
"""
from __future__ import annotations

import numpy as np

_M = np.uint64(0xFFFFFFFFFFFFFFFF)


def keep_mask(seed: int, rows: int, cols: int, p: float) -> np.ndarray:
    idx = np.arange(rows * cols, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) ^ (idx * np.uint64(0xD1B54A32D192ED03))
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        x = x ^ (x >> np.uint64(31))
    u = (x >> np.uint64(40)).astype(np.uint32)
    thresh = np.uint32(int((1.0 - float(np.float32(p))) * 16777216.0))
    return (u < thresh).reshape(rows, cols)
