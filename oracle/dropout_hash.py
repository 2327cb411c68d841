"""ORACLE (test infrastructure only) — bit-exact mirror of libgnnmp's dropout mask.

libgnnmp's fused epilogue (csrc/gemm_f32.hip: keep_elem) keeps element ``idx = row*cols + col``
(uint32 arithmetic) of a call seeded with the 64-bit ``seed`` iff
    h = fmix32((idx * 0x9E3779B1 + seed_lo) ^ seed_hi);   (h >> 8) < (uint32)((1 - (double)p) * 2^24)
where fmix32 is murmur3's finaliser and p the float32 dropout probability, and scales kept
values by 1/(1-p) — the semantics of F.dropout (src/models/gnn.py:30,51) with a counter
hash in place of torch's Philox stream.  The CPU oracle applies this exact mask so that
train-mode steps can be compared element for element.
"""
from __future__ import annotations

import numpy as np


def keep_mask(seed: int, rows: int, cols: int, p: float) -> np.ndarray:
    seed &= 0xFFFFFFFFFFFFFFFF
    idx = np.arange(rows * cols, dtype=np.uint64).astype(np.uint32)
    with np.errstate(over="ignore"):
        h = idx * np.uint32(0x9E3779B1) + np.uint32(seed & 0xFFFFFFFF)
        h = h ^ np.uint32(seed >> 32)
        h = h ^ (h >> np.uint32(16))
        h = h * np.uint32(0x85EBCA6B)
        h = h ^ (h >> np.uint32(13))
        h = h * np.uint32(0xC2B2AE35)
        h = h ^ (h >> np.uint32(16))
    thresh = np.uint32(int((1.0 - float(np.float32(p))) * 16777216.0))
    return ((h >> np.uint32(8)) < thresh).reshape(rows, cols)
