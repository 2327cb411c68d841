"""Fused SAGENet: the whole L-layer GraphSAGE forward/backward of src/models/gnn.py:35-53 as
one autograd node over libgnnmp kernels (aggregate-first, PyG's own order).

Forward, per hidden layer l (h_0 = x):
    agg_l     = mean_{j->i} h_l[j]                                   K1  (CSR gather)
    h_{l+1}   = dropout(relu([agg_l | h_l] · [W_l; W_r]ᵀ + b))      K7 NT (fused epilogue)
  the last hidden layer's epilogue also projects onto the narrow output layer
    z         = h_{L-1} · [W_l; W_r]_{L-1}ᵀ                          (registers -> [N, 2C])
    logits    = mean_{j->i} z[j, :C] + z[i, C:] + b_{L-1}            K1 narrow (8 lanes/row)
Backward:
    dz        = [meanᵀ(dlogits) | dlogits]                           K2 narrow (CSC)
    dW, db    = Gᵀ · [agg | h] with G = (dz · P) ⊙ relu'/dropout     K7 TN (G never stored)
    (deeper layers: dh = meanᵀ(G·W_l) + G·W_r via K7 NT + K2, then TN again)
Saved for backward: agg_l and h_l (the ReLU+dropout mask is h_{l+1} > 0), nothing else.

The dropout mask is a counter hash of (seed, element index) — oracle/dropout_hash.py
reproduces it bit for bit — so train-mode parity tests compare against the CPU oracle with
the very same mask.  ``F.dropout`` semantics are kept: keep with probability 1-p, scale
kept values by 1/(1-p).
"""
from __future__ import annotations

import ctypes
import functools
import os
from typing import List

import torch

from . import _lib
from .aggregation import KernelTimer, aggregate, agg_bytes
from .graph import GraphPlan, get_plan
from .planes import (BfImage, HalfPairImage, SplitImage, bf_x_image, h2_ok, is_registered, mean_planes_ok, x_padded,
                     register_input, x_image, x_only_image)

# The layer-1 operand [agg | x] as a split image (planes.py): on by default, GNNMP_PLANES=0 runs
# the in-kernel split forms instead (same results within the split's error; A/B timing).
_PLANES = os.environ.get("GNNMP_PLANES", "1") != "0"
# The 2-layer SAGE's layer-1 operand as a half-pair image (f16 hi / lo planes, 3 products: include/
# gnnmp.h gnn_split_h2_f32) rather than the split-bf16 one; GNNMP_H2=0 keeps split-bf16 (A/B).
_H2 = os.environ.get("GNNMP_H2", "1") != "0"
# GNNMP_KEEP_MASK=1: K1 also writes the half-pair NT's dropout keep bits and the NT reads them
# instead of hashing.  Off by default: measured (profiles/r18f, rocprofv3) the NT at 88.8 us with the
# bits vs 89.6 us hashing, while writing them costs K1 6.5 us (110.0 vs 103.5 us).
_KEEP_MASK = os.environ.get("GNNMP_KEEP_MASK", "0") == "1"
# The SAGE layer-0 half-pair NT's weight prep (its B image) rides in K1's launch on extra blocks
# beside the gather (gnn_sage_mean_fwd_h2 prep_b); GNNMP_K1_PREP=0 leaves it to the NT call (A/B)
_K1_PREP = os.environ.get("GNNMP_K1_PREP", "1") != "0"
# K1 gathers a zero-padded copy of the registered x (rows of col2 = 168 floats, 16-byte pieces,
# one pass per row, cached on x) instead of x itself (8-byte pieces, two passes): K1 107.0 ->
# 92.5 us, the headline step 0.3426 -> 0.3299 ms (profiles/r19n_ab.txt).  GNNMP_K1_PAD=0: A/B
_K1_PAD = os.environ.get("GNNMP_K1_PAD", "1") != "0"
# GNNMP_SIDE_PREP=1: the SAGE layer-0 NT's weight prep (the B image, latency-bound work over the
# weights only) on a side stream beside K1, joined before the NT.  Off by default: measured
# (profiles/r18h) 0.3692 vs 0.3637 ms per step in line — the captured fork / join costs more than
# the prep it hides, as in round 3
_SIDE_PREP = os.environ.get("GNNMP_SIDE_PREP", "0") == "1"
# The 2-layer SAGE backward: the layer-1 half-pair TN forms dz's meanᵀ half (the CSC sum of the CE's
# u) itself, block by block (gnn_gemm_tn_params.dz_graph, ABI 26, bit for bit), instead of a separate
# F = 2 CSC-sum launch before it; GNNMP_TN_CSC=0 keeps the separate launch (A/B)
_TN_CSC = os.environ.get("GNNMP_TN_CSC", "1") != "0"
# GCN backward: the skinny masked-gradient NT also writes its column sums (the layer below's bias
# gradient, gnn_gemm_nt_params.colsum_part) instead of a separate colsum pass; GNNMP_NT_COLSUM=0: A/B
_NT_COLSUM = os.environ.get("GNNMP_NT_COLSUM", "1") != "0"
# GCN's output aggregation and the step's masked CE in one launch (gnn_gcn_out_ce_f32) under a
# fused_ce_target; GNNMP_GCN_CE=0: A/B
_GCN_CE = os.environ.get("GNNMP_GCN_CE", "1") != "0"
# K12's backward also writes dz's column sums (the bias gradient of the conv below, SAGE-ResBN
# layer 0); GNNMP_BN_COLSUM=0: A/B
_BN_COLSUM = os.environ.get("GNNMP_BN_COLSUM", "1") != "0"
_SIDE_STREAMS = {}


def _side_stream(dev: torch.device) -> torch.cuda.Stream:
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    if key not in _SIDE_STREAMS:
        _SIDE_STREAMS[key] = torch.cuda.Stream(device=key)
    return _SIDE_STREAMS[key]

MAX_PROJ = 4  # nproj = 2 * num_classes <= 4

# K7 GEMM arithmetic (include/gnnmp.h gnn_gemm_math): "split_bf16" (default) runs every f32 operand
# as hi+mid+lo bf16 terms on the bf16 matrix cores (6 products, fp32-accurate); "f32" runs the exact
# f32 MFMA.  GNNMP_GEMM_MATH overrides the default.
GEMM_MATH = {"split_bf16": _lib.MATH_SPLIT_BF16, "f32": _lib.MATH_F32, "half_pair": _lib.MATH_HALF_PAIR}
_DEFAULT_MATH = GEMM_MATH[os.environ.get("GNNMP_GEMM_MATH", "split_bf16")]


def _math(math) -> int:
    if math is None:
        return _DEFAULT_MATH
    return GEMM_MATH[math] if isinstance(math, str) else int(math)


def _ld(t: torch.Tensor) -> int:
    return max(int(t.stride(0)), int(t.size(1)), 1)


@functools.lru_cache(maxsize=256)
def _nt_ws_bytes(n, k1, k2) -> int:
    nb = _lib.c_size(0)
    _lib.call("gnn_gemm_nt_workspace_size", n, k1, k2, nb)
    return int(nb.value)


@functools.lru_cache(maxsize=256)
def _tn_ws_bytes(M, nr, kc, nproj) -> int:
    nb = _lib.c_size(0)
    _lib.call("gnn_gemm_tn_workspace_size", M, nr, kc, nproj, nb)
    return int(nb.value)


def _nt_workspace(device, n, k1, k2):
    return torch.empty(max(_nt_ws_bytes(n, k1, k2) // 4, 1), dtype=torch.float32, device=device)


def _planes_fields(planes):
    if planes is None:
        return (None, 0, 0, 0, _lib.PLANES_SPLIT_BF16)
    return (planes.ptr, planes.ld, planes.ps, planes.col2, getattr(planes, "fmt", _lib.PLANES_SPLIT_BF16))


# bf16 storage: layer operands as one-plane bf16 images (planes.BfImage) for the weight-stationary
# bf16 NT; GNNMP_BF_IMAGE=0 keeps the tiled bf16 NT over separate A1 / A2 (A/B timing)
_BF_IMAGE = os.environ.get("GNNMP_BF_IMAGE", "1") != "0"


def h2s_nt_ok(n: int, k1: int, k2: int, dtype=torch.float32) -> bool:
    """Whether a w1/w2-form NT with math="half_pair" runs the in-kernel half-pair kernel (gemm_x3.hip
    nt_h2s_ok; the skinny VALU shapes, n <= 8 or k <= 8, keep their own kernels): the shapes a
    ``row_exp`` may be asked of."""
    return dtype == torch.float32 and 8 < n <= 128 and k1 % 16 == 0 and k2 % 16 == 0 and 16 <= k1 + k2 <= 128


def gemm_nt(a1, bt, n, a2=None, bias=None, relu=False, dropout_p=0.0, seed=0, proj=None, z=None,
            out=None, want_c=True, seed_ptr=None, w1=None, w2=None, math=None, mask=None, mask_scale=1.0,
            planes=None, check_planes=False, keep_mask=None, workspace=None, b_stage=None, colsum=False,
            row_exp=None):
    """C = epilogue([a1 | a2] · B) on the NT kernels; B = bt ([K, n] row-major) or, with bt None,
    [w1 | w2]ᵀ read in place from PyTorch Linear weights w1 [n, k1], w2 [n, k2].
    bf16 A (the bf16-storage path) needs the w1/w2 form; C is then bf16 too.
    ``planes`` (planes.SplitImage): A read from the split image; a1 / a2 may then be None.
    ``check_planes``: only report whether the call would take the split-image kernel (no launch).
    ``keep_mask`` (half-pair planes with dropout): the keep bits K1 wrote for this call's seed.
    ``b_stage`` (image-A forms, with an explicit ``workspace``): "prep" launches only the B-image
    prep (gnn_gemm_nt_prep_b; returns None), "ready" only the GEMM over the image a "prep" call of
    the same weights left in ``workspace``; "params" launches nothing and returns the call's
    GnnGemmNTParams (K1's prep_b: HalfPairImage.fill_mean).
    ``colsum``: also return Σ_rows C ([n] f32) — on the skinny-K form its blocks write the column
    sums as they store C (gnn_gemm_nt_params.colsum_part) and one small launch adds them
    (gnn_colsum_finish_f32); otherwise a gnn_colsum_f32 pass over C.  Returns (C, Σ C).
    ``row_exp`` (int32 [M], math="half_pair", the shapes of h2s_nt_ok): receives the per-row
    exponents of [a1 | a2] for a half-pair TN over the same operand (gemm_tn(row_exp=...))."""
    if planes is not None:
        M, k1, k2, dev = planes.n, planes.k1, planes.k2, planes.img.device
    else:
        M, k1, k2, dev = a1.size(0), a1.size(1), (a2.size(1) if a2 is not None else 0), a1.device
    bf = getattr(planes, "bf16", False) or (a1 is not None and a1.dtype == torch.bfloat16)
    if out is None and want_c and not check_planes and b_stage not in ("prep", "params"):
        out = torch.empty((M, n), dtype=torch.bfloat16 if bf else torch.float32, device=dev)
    ws = workspace
    if ws is None and w1 is not None:  # B pre-split image for the streaming split-bf16 kernel (≈24 KB per 32 of K)
        ws = _nt_workspace(dev, n, k1, k2)
    p = _lib.GnnGemmNTParams(
        M, n,
        _lib.ptr(a1), _ld(a1) if a1 is not None else 0, k1,
        _lib.ptr(a2), _ld(a2) if a2 is not None else 0, k2,
        _lib.ptr(bt), _ld(bt) if bt is not None else 0,
        _lib.ptr(w1), _lib.ptr(w2), _ld(w1) if w1 is not None else 0, _ld(w2) if w2 is not None else 0,
        _lib.ptr(out), _ld(out) if out is not None else 0,
        _lib.ptr(bias), int(relu), float(dropout_p), int(seed) & 0xFFFFFFFFFFFFFFFF, _lib.ptr(seed_ptr),
        _lib.ptr(proj), proj.size(0) if proj is not None else 0, _lib.ptr(z), _ld(z) if z is not None else 0,
        _math(math),
        _lib.ptr(ws), ws.numel() * 4 if ws is not None else 0,
        _lib.DTYPE_BF16 if bf else _lib.DTYPE_F32,
        _lib.DTYPE_BF16 if (out is not None and out.dtype == torch.bfloat16) else _lib.DTYPE_F32,
        _lib.ptr(mask), _ld(mask) if mask is not None else 0, float(mask_scale),
        *_planes_fields(planes), _lib.ptr(keep_mask), int(b_stage == "ready"),
        int(getattr(planes, "exp", 0)),
    )
    if row_exp is not None:
        p.row_exp = row_exp.data_ptr()
    part = None
    if colsum and out is not None and b_stage is None and not check_planes:
        nb = ctypes.c_int32(0)
        _lib.call("gnn_gemm_nt_colsum_blocks", p, ctypes.byref(nb))
        if nb.value > 0:
            part = torch.empty(nb.value * n, dtype=torch.float32, device=dev)
            p.colsum_part, p.colsum_cap = part.data_ptr(), part.numel()
    if check_planes:
        return bool(_lib.load().gnn_gemm_nt_planes_ok(p))
    if b_stage == "params":
        return p
    if b_stage == "prep":
        _lib.call("gnn_gemm_nt_prep_b", p, _lib.stream_handle(dev))
        return None
    if KernelTimer.active:
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
    _lib.call("gnn_gemm_nt_f32", p, _lib.stream_handle(dev))
    if KernelTimer.active:
        e1.record()
        k = k1 + k2
        # tag: kind, M, K, N, A element bytes, C element bytes, MFMA products per bf16 term
        # (6 split-bf16, 1 bf16 storage, 0 exact f32, -1 the VALU kernels of the skinny shapes).
        # A split image is priced at the algorithmic f32 bytes; it moves 6 B / element.
        ea = 2 if bf else (4 if a1 is None else a1.element_size())
        prod = 0 if (_math(math) == _lib.MATH_F32 or w1 is None) else (1 if ea == 2 else 6)
        if getattr(planes, "fmt", None) == _lib.PLANES_HALF_PAIR or (
                _math(math) == _lib.MATH_HALF_PAIR and planes is None and h2s_nt_ok(n, k1, k2, a1.dtype)):
            prod = 3  # f16 half-pair: 3 products
        if ea == 4 and proj is None and (n <= 8 or (k <= 8 and a2 is None)):
            prod = -1
        KernelTimer.records.append((("gemm_nt", M, k, n, ea, out.element_size() if out is not None else 0, prod),
                                    e0, e1, 2 * M * k * n))
    if colsum:
        from .aggregation import colsum as _colsum

        if part is None:
            return out, _colsum(out)
        db = torch.empty(n, dtype=torch.float32, device=dev)
        _lib.call("gnn_colsum_finish_f32", part.data_ptr(), part.numel() // n, n, db.data_ptr(), _lib.stream_handle(dev))
        return out, db
    return out


def gemm_tn(nr, a1, a2=None, g=None, dz=None, proj=None, h=None, hscale=1.0, gout=None, math=None,
            planes=None, check_planes=False, sq=None, sq_skip=(0, 0), row_exp=None, csc=None):
    """((Gᵀ·a1, Gᵀ·a2), db, dzᵀ·h, dzsum) from one flat fp32 buffer — the MFMA TN kernel.
    ``planes``: A read from a split image (a1 / a2 may be None); ``check_planes`` as gemm_nt.
    ``sq`` = (partials buffer, step tensor) of train_ops.grad_sq_request: the reduce also writes
    the clip + Adam norm partials of the output outside ``sq_skip`` (indices into the flat output,
    negative ones from its end), recorded by train_ops.grad_sq_produced.
    ``row_exp``: the int32 row exponents a half-pair NT wrote for [a1 | a2]; with math="half_pair"
    and the plain g form the TN then runs in half-pair arithmetic (gnn_gemm_tn_params.row_exp).
    ``csc`` = (plan, u): the half-pair dz-form TN forms dz[:, :u.size(1)] itself as the transposed
    SUM of u over the plan (gnn_gemm_tn_params.dz_graph, ABI 26) instead of reading it."""
    if planes is not None:
        M, k1, k2, dev = planes.n, planes.k1, planes.k2, planes.img.device
    else:
        M, k1, k2, dev = a1.size(0), a1.size(1), (a2.size(1) if a2 is not None else 0), a1.device
    bf = getattr(planes, "bf16", False) or (a1 is not None and a1.dtype == torch.bfloat16)
    nproj = proj.size(0) if dz is not None else 0
    n_out = nr * (k1 + k2) + nr + nproj * nr + nproj
    p = _lib.GnnGemmTNParams(
        M, nr,
        _lib.ptr(g), _ld(g) if g is not None else 0,
        _lib.ptr(dz), _ld(dz) if dz is not None else 0,
        _lib.ptr(proj), nproj,
        _lib.ptr(h), _ld(h) if h is not None else 0, float(hscale),
        _lib.ptr(gout), _ld(gout) if gout is not None else 0,
        _lib.ptr(a1), _ld(a1) if a1 is not None else 0, k1,
        _lib.ptr(a2), _ld(a2) if a2 is not None else 0, k2,
        _math(math),
        _lib.DTYPE_BF16 if bf else _lib.DTYPE_F32,
        _lib.DTYPE_BF16 if (h is not None and h.dtype == torch.bfloat16) else _lib.DTYPE_F32,
        *_planes_fields(planes),
        _lib.DTYPE_BF16 if any(t is not None and t.dtype == torch.bfloat16 for t in (g, gout)) else _lib.DTYPE_F32,
        int(getattr(planes, "exp", 0)),
    )
    if row_exp is not None:
        p.row_exp = row_exp.data_ptr()
    if g is not None and dz is None and planes is not None:
        from .aggregation import rowmax_of

        rm = rowmax_of(g)  # the producer's max |g| per 16-row group (ABI 25): no scan pass in the TN
        if rm is not None:
            p.g_rowmax = rm.data_ptr()
    if csc is not None:
        cplan, u = csc
        p.dz_graph, p.dz_u, p.ldu, p.dz_cols = ctypes.addressof(cplan.c_graph), u.data_ptr(), _ld(u), u.size(1)
    if check_planes:
        return bool(_lib.load().gnn_gemm_tn_planes_ok(p))
    out = torch.empty(n_out, dtype=torch.float32, device=dev)
    if sq is not None:
        lo, hi = (int(v) + n_out if v < 0 else int(v) for v in sq_skip)
        p.sq_partial, p.sq_step = sq[0].data_ptr(), sq[1].data_ptr()
        p.sq_skip_lo, p.sq_skip_hi, p.sq_cap = lo, hi, sq[0].numel()
    ws = torch.empty(max(_tn_ws_bytes(M, nr, k1 + k2, nproj) // 4, 1), dtype=torch.float32, device=dev)
    if KernelTimer.active:
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
    _lib.call("gnn_gemm_tn_f32", p, out.data_ptr(), ws.data_ptr(), ws.numel() * 4, _lib.stream_handle(dev))
    if sq is not None:
        from .train_ops import grad_sq_produced

        # out._version: the gradients are views of out (AccumulateGrad adopts them detached, sharing
        # its version counter), so any in-place edit between here and ClipAdam.step — GradScaler's
        # unscale_, a mul_, an all-reduce — bumps it and voids the fold
        grad_sq_produced(dev, (out, n_out, (lo, hi), _sq_blocks(n_out), sq[0], sq[1], out._version))
    if KernelTimer.active:
        e1.record()
        ea = 2 if bf else (4 if a1 is None else a1.element_size())
        prod = 0 if _math(math) == _lib.MATH_F32 else (1 if ea == 2 else 6)
        if getattr(planes, "fmt", None) == _lib.PLANES_HALF_PAIR or (
                _math(math) == _lib.MATH_HALF_PAIR and row_exp is not None and g is not None and dz is None):
            prod = 3
        if ea == 4 and nr <= 8 and dz is None and h is None and gout is None:
            prod = -1
        KernelTimer.records.append((("gemm_tn", M, k1 + k2, nr, ea, h.element_size() if h is not None else 4, prod),
                                    e0, e1, 2 * M * (k1 + k2) * nr))
    o = 0
    dW1 = out[o: o + nr * k1].view(nr, k1)  # contiguous per segment: autograd adopts them, no clone
    o += nr * k1
    dW2_ = out[o: o + nr * k2].view(nr, k2) if k2 else None
    o += nr * k2
    db = out[o: o + nr]
    o += nr
    dW2 = out[o: o + nproj * nr].view(nproj, nr) if nproj else None
    o += nproj * nr
    dzs = out[o: o + nproj] if nproj else None
    return (dW1, dW2_), db, dW2, dzs


@functools.lru_cache(maxsize=64)
def _sq_blocks(n_out: int) -> int:
    nb = _lib.c_i32(0)
    _lib.call("gnn_gemm_tn_sq_blocks", n_out, ctypes.byref(nb))
    return int(nb.value)


def gemm_nt_input(x: torch.Tensor, n: int, **kw):
    """gemm_nt(x, None, n, **kw) (w1 form, no a2) for a layer whose A operand is the model input x:
    on the split-image NT over x's cached planes (planes.x_only_image) when it takes the shape."""
    if _H2:  # the half-pair image (3 products) when x fits it
        im = x_only_image(x, HalfPairImage)
        if im is not None and gemm_nt(None, None, n, planes=im, check_planes=True, **kw):
            return gemm_nt(None, None, n, planes=im, **kw)
    im = x_only_image(x)
    if im is not None and gemm_nt(None, None, n, planes=im, check_planes=True, **kw):
        return gemm_nt(None, None, n, planes=im, **kw)
    return gemm_nt(x, None, n, **kw)


def _csc_fold(ctx, dz, u, hscale):
    """(plan, u) when the 2-layer SAGE backward's one TN (layer 1, half-pair image, dz form, no input
    gradient) takes the folded CSC sum of u (ABI 26), else None (the caller runs the CSC sum)."""
    L = ctx.meta[0]
    if not _TN_CSC or L != 2 or ctx.needs_input_grad[0] or ctx.bimgs[0] is not None:
        return None
    saved = ctx.saved_tensors
    if saved[L] is not None or getattr(ctx, "image", None) is None or not isinstance(ctx.image[0], HalfPairImage):
        return None  # layer 1 not on the half-pair image of [agg | x]
    im = ctx.image[0]
    hs1, Wl0 = saved[1], saved[2 * L - 1]
    csc = (ctx.plan, u)
    if not gemm_tn(Wl0.size(0), None, None, h=hs1, hscale=hscale, planes=im, check_planes=True, dz=dz, proj=ctx.P,
                   csc=csc):
        return None
    return csc


def gemm_tn_input(nr: int, x: torch.Tensor, g: torch.Tensor):
    """gemm_tn(nr, x, g=g) for a layer whose A operand is the model input x: on the half-pair TN
    over x's cached half-pair image (the one the forward NT read: 4 B per element, 3 products)
    when it takes the shape, else the split-image TN over x's split-bf16 planes, else the f32 form."""
    if _H2:
        im = x_only_image(x, HalfPairImage)
        if im is not None and gemm_tn(nr, None, g=g, planes=im, check_planes=True):
            return gemm_tn(nr, None, g=g, planes=im)
    im = x_only_image(x)
    if im is not None and gemm_tn(nr, None, g=g, planes=im, check_planes=True):
        return gemm_tn(nr, None, g=g, planes=im)
    return gemm_tn(nr, x, g=g)


def _layer0_image(x: torch.Tensor, n_out: int, nt_kw, h2: bool = False):
    """The split image of [agg | x] when the planes path takes this layer (else None): x must be a
    registered constant input (planes.register_input) — its planes are built once and reused; a
    per-batch or per-step input keeps the in-kernel split (gemm_nt over f32 [agg | x]).
    h2: prefer the half-pair image (f16 hi / lo planes, 3 products) when x fits it (finite)
    — the 2-layer net, whose layer-0 weight gradient is the TN's dz form."""
    if not (_PLANES and is_registered(x) and mean_planes_ok(x)) or x.size(0) < 32:
        return None
    if h2 and _H2 and HalfPairImage.addressable(x.size(0), x.size(1), x.size(1)) and h2_ok(x):
        im = x_image(x, HalfPairImage)
        if gemm_nt(None, None, n_out, planes=im, check_planes=True, **nt_kw):
            return im
    if not SplitImage.addressable(x.size(0), x.size(1), x.size(1)):
        return None
    im = x_image(x)
    if not gemm_nt(None, None, n_out, planes=im, check_planes=True, **nt_kw):
        return None
    return im


def _bf_image0(x: torch.Tensor, L: int, Wl):
    """The cached layer-0 bf16 image when every hidden layer's NT can run on images (the shapes
    nt_img16_ok takes: image rows of 256 or 336 columns, 8 <= F_out <= 128 with F_out % 8 == 0,
    31-bit byte offsets), else None (the tiled bf16 NT over separate operands)."""
    if not _BF_IMAGE or L < 2 or x.dim() != 2 or x.size(0) < 32 or x.stride(1) != 1:
        return None
    n, fi = x.size(0), x.size(1)
    for l in range(L - 1):
        fo = Wl[l].size(0)
        ld = ((fi + 7) // 8 * 16 + 15) // 16 * 16
        if ld not in (256, 336) or not (8 <= fo <= 128 and fo % 8 == 0):
            return None
        if n * max(ld, fo) * 2 >= 2 ** 31 or n * 4 * 4 >= 2 ** 31:
            return None
        fi = fo
    return bf_x_image(x)


class _FusedSAGE(torch.autograd.Function):
    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.float32)
    def forward(ctx, x, plan: GraphPlan, dropout_p: float, seeds: List[int], seed_ctr, P, *params):
        # x bf16 selects the bf16-storage path: agg_l and h_l stored bf16, GEMMs on bf16 operands
        # (weights rounded to bf16) with f32 accumulation; z, logits and all gradients stay f32.
        # P: [W_l ; W_r] of the output layer, [2C, F_{L-1}] (sage_forward's _output_weights)
        L = len(params) // 3
        Wl = params[0::3]
        bl = params[1::3]
        Wr = params[2::3]
        x = x.contiguous()
        C = Wl[-1].size(0)
        train_drop = dropout_p if dropout_p > 0 else 0.0
        hs = [x]
        aggs = []
        z = None
        ctx.image = None
        bim = _bf_image0(x, L, Wl) if x.dtype == torch.bfloat16 else None
        ctx.bimgs = [None] * (L - 1)
        for l in range(L - 1):
            h = hs[-1]
            last_hidden = l == L - 2
            if last_hidden:
                z = torch.empty((h.size(0), 2 * C), dtype=torch.float32, device=h.device)
            # B = [W_l | W_r]ᵀ read in place from the Linear weights (K-contiguous [n][k] rows are
            # the NT kernel's LDS image): no transposed copy
            nt_kw = dict(w1=Wl[l], w2=Wr[l], bias=bl[l], relu=True, dropout_p=train_drop, seed=seeds[l],
                         proj=P if last_hidden else None, z=z if last_hidden else None, seed_ptr=seed_ctr)
            if bim is not None:  # bf16 storage on images: K1 into A1, the NT's C into the next image's A2
                fo = Wl[l].size(0)
                nxt = BfImage(h.size(0), fo, fo, h.device) if not last_hidden else None
                out = nxt.a2 if nxt is not None else torch.empty((h.size(0), fo), dtype=torch.bfloat16,
                                                                  device=h.device)
                if _K1_PAD and bim.k2 == bim.k1 < bim.col2 and bim.col2 % 4 == 0 and bim.ld >= 2 * bim.col2:
                    # h is the image's A2 half, zero columns up to ld (a padded image is zero-
                    # allocated): gather it there at the padded width, 8-byte pieces in one pass
                    # per row; the padding columns aggregate to the zeros already in A1's
                    aggregate(plan, bim.img[:, bim.col2: 2 * bim.col2], _lib.AGG_MEAN, nodew=plan.deg,
                              out=bim.img[:, : bim.col2])
                else:
                    aggregate(plan, h, _lib.AGG_MEAN, nodew=plan.deg, out=bim.a1)
                hn = gemm_nt(None, None, fo, planes=bim, out=out, **nt_kw)
                ctx.bimgs[l] = bim
                aggs.append(bim.a1)
                hs.append(hn)
                bim = nxt
                continue
            im = _layer0_image(h, Wl[0].size(0), nt_kw, h2=last_hidden) if l == 0 else None
            if im is not None:  # agg written straight into the split image by K1; A staged as planes
                keep = None
                if isinstance(im, HalfPairImage) and train_drop > 0 and _KEEP_MASK:  # K1 also writes the NT's keep bits
                    kb = im.keep_buffer()
                    keep = (kb, Wl[l].size(0), train_drop, seeds[l], seed_ctr)
                    nt_kw = dict(nt_kw, keep_mask=kb)
                n_out = Wl[l].size(0)
                ws, side, ready = _nt_workspace(h.device, n_out, im.k1, im.k2), None, False
                prep_b = None
                if _K1_PREP and isinstance(im, HalfPairImage):  # the B prep inside K1's launch
                    prep_b = gemm_nt(None, None, n_out, planes=im, workspace=ws, b_stage="params", **nt_kw)
                    ready = True
                elif _SIDE_PREP:  # the B prep beside K1 on a side stream (it reads only the weights)
                    side, cur = _side_stream(h.device), torch.cuda.current_stream(h.device)
                    side.wait_stream(cur)
                    with torch.cuda.stream(side):
                        gemm_nt(None, None, n_out, planes=im, workspace=ws, b_stage="prep", **nt_kw)
                    ready = True
                xp = x_padded(h, im.col2) if _K1_PAD and im.col2 % 4 == 0 and im.col2 > h.size(1) else None
                ctx.image = (im, im.fill_mean(plan, h, keep, prep_b=prep_b, x_pad=xp))
                if side is not None:
                    cur.wait_stream(side)
                hn = gemm_nt(None, None, n_out, planes=im, workspace=ws, b_stage="ready" if ready else None, **nt_kw)
                agg = None
            else:
                agg = aggregate(plan, h, _lib.AGG_MEAN, nodew=plan.deg)
                hn = gemm_nt(agg, None, Wl[l].size(0), a2=h, **nt_kw)
            aggs.append(agg)
            hs.append(hn)
        from .train_ops import ce_target, sage_out_mean_ce

        tgt = ce_target()
        if tgt is not None and any(ctx.needs_input_grad) and z.dtype == torch.float32 and C <= 4:
            # the step's masked CE in the output mean's launch (train_ops.fused_ce_target)
            e0 = KernelTimer.begin()
            logits, ce = sage_out_mean_ce(plan, z, C, bl[-1], tgt)
            KernelTimer.end(e0, ("agg", _lib.AGG_MEAN, False, C), agg_bytes(plan, C, _lib.AGG_MEAN, False, False))
            logits._gnnmp_ce = ce
        else:
            logits = aggregate(plan, z[:, :C], _lib.AGG_MEAN, nodew=plan.deg, addend=z[:, C:], bias=bl[-1])
        ctx.plan = plan
        ctx.meta = (L, C, float(dropout_p))
        ctx.P = P  # the output layer's stacked weights, reused by the backward (no second cat)
        ctx.save_for_backward(*hs, *aggs, *params)
        return logits

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, dlogits):
        plan = ctx.plan
        L, C, p = ctx.meta
        saved = ctx.saved_tensors
        hs = saved[:L]
        aggs = saved[L: 2 * L - 1]
        params = saved[2 * L - 1:]
        Wl, Wr = params[0::3], params[2::3]
        hscale = 1.0 / (1.0 - p) if p > 0 else 1.0
        N = dlogits.size(0)
        csc_fold = None  # (plan, u) when the layer's TN forms dz's meanᵀ half itself (ABI 26)
        buf = getattr(dlogits, "_gnnmp_dz", None)  # the fused CE's [N, 2C] buffer, dlogits its right half
        if (buf is not None and buf.shape == (N, 2 * C) and dlogits.stride() == (2 * C, 1)
                and dlogits.data_ptr() == buf.data_ptr() + C * buf.element_size()):
            dz = buf
            u = getattr(dlogits, "_gnnmp_u", None)  # dlogits / max(deg, 1) from the forward's CE launch
            if u is not None:  # meanᵀ as a plain CSC sum: MEAN_BWD's per-slot terms precomputed, same bits
                csc_fold = _csc_fold(ctx, dz, u, hscale)
                if csc_fold is None:
                    aggregate(plan, u, _lib.AGG_SUM, transpose=True, out=dz[:, :C])
            else:
                aggregate(plan, dlogits, _lib.AGG_MEAN_BWD, transpose=True, nodew=plan.deg, out=dz[:, :C])
        else:
            dlogits = dlogits.contiguous()
            dz = torch.empty((N, 2 * C), dtype=torch.float32, device=dlogits.device)
            aggregate(plan, dlogits, _lib.AGG_MEAN_BWD, transpose=True, nodew=plan.deg, out=dz[:, :C])
            dz[:, C:].copy_(dlogits)
        P = ctx.P
        grads = [None] * (3 * L)
        need_x = ctx.needs_input_grad[0]
        from .train_ops import grad_sq_produced, grad_sq_request

        grad_sq_produced(dz.device, None)
        # 2 layers: the one TN below writes every parameter's gradient (dzsum[:C], Σ meanᵀ(dlogits),
        # is not one of them) — Σg² for clip_grad_norm_ comes with its reduce.  Only on the
        # unit-gradient path (dz is the CE's tagged buffer: loss.backward(unit_gradient)): a scaled
        # loss (GradScaler) hands its gradients to unscale_, which rewrites them in place without
        # bumping their version counter, so its Σg² must be read after that, by ClipAdam's own pass
        sq = grad_sq_request(dz.device) if (L == 2 and dz is buf) else None
        g = None
        for l in range(L - 2, -1, -1):
            fo, fi = Wl[l].shape
            need_g = l > 0 or need_x
            bim = ctx.bimgs[l]
            # bf16 storage: G and the input gradient dh stay bf16 between the layers (autocast's
            # rounding points): the TN writes the rounded G into the right half of a [meanᵀ(G) | G]
            # bf16 image, whose left half the bf16 transposed aggregation fills; dh is then ONE
            # one-product bf16 image NT.  (Needs fo <= 128 and fi <= 128 with the image's widths.)
            gimg = None
            if bim is not None and need_g and fi <= 128 and 8 <= fi and fi % 8 == 0 and 2 * fo in (256,) and _BF_IMAGE:
                gimg = BfImage(N, fo, fo, dz.device)
                gout = gimg.a2
            else:
                gout = torch.empty((N, fo), dtype=torch.float32, device=dz.device) if need_g else None
            a_l, im = aggs[l], None
            if bim is not None:  # bf16 storage: the TN reads the layer's bf16 image
                tn_kw = dict(dz=dz, proj=P) if l == L - 2 else dict(g=g)
                if gemm_tn(fo, None, None, h=hs[l + 1], hscale=hscale, gout=gout, planes=bim, check_planes=True,
                           **tn_kw):
                    im = bim
            if a_l is None:  # layer 0 on the split image (refreshed if another forward reused it)
                im, gen = ctx.image
                if im.gen != gen:
                    im.fill_mean(plan, hs[0])
                tn_kw = dict(dz=dz, proj=P) if l == L - 2 else dict(g=g)
                if not gemm_tn(fo, None, None, h=hs[l + 1], hscale=hscale, gout=gout, planes=im,
                               check_planes=True, **tn_kw):
                    a_l, im = aggregate(plan, hs[0], _lib.AGG_MEAN, nodew=plan.deg), None
            if l == L - 2:
                dW, db, dW2, dzs = gemm_tn(fo, a_l, hs[l], dz=dz, proj=P, h=hs[l + 1], hscale=hscale,
                                           gout=gout, planes=im, sq=sq, sq_skip=(-2 * C, -C), csc=csc_fold)
                grads[3 * (L - 1) + 0] = dW2[:C]
                grads[3 * (L - 1) + 1] = dzs[C:]
                grads[3 * (L - 1) + 2] = dW2[C:]
            else:
                dW, db, _, _ = gemm_tn(fo, a_l, hs[l], g=g, h=hs[l + 1], hscale=hscale, gout=gout, planes=im)
            grads[3 * l + 0] = dW[0]
            grads[3 * l + 1] = db
            grads[3 * l + 2] = dW[1]
            if gimg is not None:
                aggregate(plan, gout, _lib.AGG_MEAN_BWD, transpose=True, nodew=plan.deg, out=gimg.a1)
                g = gemm_nt(None, None, fi, planes=gimg, w1=Wl[l].t().contiguous(), w2=Wr[l].t().contiguous(),
                            out=torch.empty((N, fi), dtype=torch.bfloat16, device=dz.device))
            elif need_g and fi <= 128:
                # dh_l = meanᵀ(G · W_l) + G · W_r = [meanᵀ(G) | G] · [W_l; W_r]  (G = dL/dpre_{l+1}):
                # reassociated so one transposed aggregation of G (width fo) and ONE GEMM
                # (K = 2·fo, split-bf16, W read as the [fi, fo] transposes) replace two GEMMs
                # and the [N, 2·fi] intermediate
                aggG = aggregate(plan, gout, _lib.AGG_MEAN_BWD, transpose=True, nodew=plan.deg)
                g = gemm_nt(aggG, None, fi, a2=gout, w1=Wl[l].t().contiguous(), w2=Wr[l].t().contiguous())
            elif need_g:
                # fi > 128 (the input layer's dx): W [fo, fi] is already the row-major [K, N]
                # operand of the NT kernel (exact f32 form)
                dA = torch.empty((N, 2 * fi), dtype=torch.float32, device=dz.device)
                gemm_nt(gout, Wl[l], fi, out=dA[:, :fi])
                gemm_nt(gout, Wr[l], fi, out=dA[:, fi:])
                g = aggregate(plan, dA[:, :fi], _lib.AGG_MEAN_BWD, transpose=True, nodew=plan.deg,
                              addend=dA[:, fi:])
            # g: next (lower) layer's upstream gradient w.r.t. h_l, masked inside its TN
        dx = g.to(hs[0].dtype) if need_x else None
        return (dx, None, None, None, None, None, *grads)


class _FusedGCN(torch.autograd.Function):
    """GCNNet (src/models/gnn.py:14-32) as one autograd node, transform first (PyG's order):

        y_l      = h_l · W_lᵀ                               K7 NT (w1 form, weight in place)
        h_{l+1}  = dropout(relu(Â y_l + b_l))               K4 CSR, bias / ReLU / counter-hash
                                                            dropout in the aggregation's store
        logits   = Â (h_{L-1} · W_{L-1}ᵀ) + b_{L-1}         K7 skinny NT + K4 (bias)
    Backward, layer by layer from the top (g = dL/d(Â y + b), g_top = dlogits):
        dy = Âᵀ g (K4 CSC),  db = Σ_rows g,  dW = dyᵀ · h_l (K7 TN)
        g_below = (dy · W_l) ⊙ [h_l > 0] / (1 − p)          skinny NT with the mask epilogue
    (h_l > 0 exactly where ReLU passed and dropout kept).  Saved: the layer inputs h_l only;
    no torch elementwise kernels on the path."""

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.float32)
    def forward(ctx, x, plan: GraphPlan, dropout_p: float, seeds: List[int], seed_ctr, *params):
        L = len(params) // 2
        W, b = params[0::2], params[1::2]
        hs = [x.contiguous()]
        dinv = plan.dinv
        for l in range(L - 1):
            y = gemm_nt_input(hs[0], W[0].size(0), w1=W[0]) if l == 0 else gemm_nt(hs[-1], None, W[l].size(0), w1=W[l])
            hs.append(aggregate(plan, y, _lib.AGG_GCN, nodew=dinv, bias=b[l], relu=True,
                                dropout_p=dropout_p, seed=seeds[l], seed_ptr=seed_ctr))
        y = gemm_nt(hs[-1], None, W[-1].size(0), w1=W[-1])
        from .train_ops import ce_target, gcn_out_ce

        tgt = ce_target()
        if tgt is not None and any(ctx.needs_input_grad) and y.dtype == torch.float32 and y.size(1) <= 2 \
                and y.size(0) > 0 and _GCN_CE:
            # the step's masked CE in the output aggregation's launch (train_ops.fused_ce_target)
            e0 = KernelTimer.begin()
            logits, ce = gcn_out_ce(plan, y, b[-1], tgt)
            KernelTimer.end(e0, ("agg", _lib.AGG_GCN, False, y.size(1)), agg_bytes(plan, y.size(1), _lib.AGG_GCN, False, False))
            logits._gnnmp_ce = ce
        else:
            logits = aggregate(plan, y, _lib.AGG_GCN, nodew=dinv, bias=b[-1])
        ctx.plan = plan
        ctx.meta = (L, float(dropout_p))
        ctx.save_for_backward(*hs, *params)
        return logits

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, dlogits):
        from .aggregation import colsum_of

        plan = ctx.plan
        L, p = ctx.meta
        saved = ctx.saved_tensors
        hs, params = saved[:L], saved[L:]
        W = params[0::2]
        scale = 1.0 / (1.0 - p) if p > 0 else 1.0
        dinv = plan.dinv
        grads = [None] * (2 * L)
        # the fused CE's dlogits is the right half of its [N, 2C] buffer: read in place (row stride 2C)
        g = dlogits if (dlogits.dim() == 2 and dlogits.stride(1) == 1 and dlogits.stride(0) >= dlogits.size(1)) \
            else dlogits.contiguous()
        dx = None
        db_next = None  # Σ_rows g of the layer below, from the skinny NT that wrote g
        for l in range(L - 1, -1, -1):
            dy = aggregate(plan, g, _lib.AGG_GCN, transpose=True, nodew=dinv)
            grads[2 * l + 1] = db_next if db_next is not None else colsum_of(g)
            db_next = None
            (dW, _), _, _, _ = gemm_tn_input(W[l].size(0), hs[l], dy) if l == 0 else gemm_tn(W[l].size(0), hs[l], g=dy)
            grads[2 * l] = dW
            fo, fi = W[l].shape
            if l > 0:  # W [fo, fi] is the row-major [K, N] operand of dh = dy · W
                if (fo <= 8 or fi <= 8) and _NT_COLSUM:  # (its column sums: the next layer's bias gradient)
                    g, db_next = gemm_nt(dy, W[l], fi, mask=hs[l], mask_scale=scale, colsum=True)
                elif fo <= 8 or fi <= 8:
                    g = gemm_nt(dy, W[l], fi, mask=hs[l], mask_scale=scale)
                else:
                    g = gemm_nt(dy, W[l], fi)
                    g.mul_((hs[l] > 0).to(g.dtype) * scale)
            elif ctx.needs_input_grad[0]:
                dx = gemm_nt(dy, W[l], fi)
        return (dx, None, None, None, None, *grads)


def gcn_fusable(model) -> bool:
    """GCNNet of GCNConv(bias) layers within the kernels' widths, not in explain mode."""
    convs = list(model.convs)
    if len(convs) < 2:
        return False
    for c in convs:
        if getattr(c, "explain", False) or c.bias is None:
            return False
        if c.out_channels > 128 or c.in_channels > 384:
            return False
    return True


def gcn_forward(model, x: torch.Tensor, edge_index: torch.Tensor) -> torch.Tensor:
    plan = get_plan(edge_index, x.size(0), _lib.LOOPS_REPLACE)
    L = len(model.convs)
    p = float(model.dropout) if model.training else 0.0
    seeds, ctr = dropout_seeds(L, p, x)
    params = []
    for c in model.convs:
        params += [c.lin.weight, c.bias]
    return _FusedGCN.apply(x, plan, p, seeds, ctr, *params)


def fusable(model) -> bool:
    """SAGENet with narrow output (2·classes <= 4), widths within the fused kernels' limits."""
    convs = list(model.convs)
    if len(convs) < 2:
        return False
    for c in convs:
        if getattr(c, "explain", False):  # explain mode: per-conv path with the edge mask
            return False
        if getattr(c, "aggr", None) != "mean" or c.lin_l.bias is None:
            return False
    for c in convs[:-1]:
        if c.out_channels > 128 or 2 * c.in_channels > 384:
            return False
    return 2 * convs[-1].out_channels <= MAX_PROJ and convs[-1].in_channels <= 128


_SEED_CTR = {}


def _graph_seed_counter(device: torch.device) -> torch.Tensor:
    """Per-device int64 dropout counter for HIP-graph capture.

    Eager calls draw fresh seeds from torch's CPU generator (respects torch.manual_seed).  Under
    stream capture a host-drawn seed would be frozen into the graph, so the forward instead
    bumps this device counter (an add_ recorded in the graph) and the kernel derives the
    seed from it on every replay.
    """
    c = _SEED_CTR.get(device)
    if c is None:  # a fill kernel (capture-safe); start value from the seed without consuming the RNG
        c = torch.full((1,), (torch.initial_seed() * 0x9E3779B97F4A7C15 + 1) % (2 ** 62), dtype=torch.int64,
                       device=device)
        _SEED_CTR[device] = c
    return c


# Inside train_gnn.CapturedStep two pieces of end-of-step work can be deferred to the step's end:
# the dropout counter's per-step bump (always: nothing in a step reads the counter after its
# forward) and — only with CapturedStep(defer_loss=True) — the fused CE's loss scalar.  ClipAdam's
# launch carries both (gnn_adam_group.bump_counter / loss_partial) — two launches fewer per
# replayed step — or, with another optimizer, CapturedStep records them itself at the end of the
# capture.  The loss deferral is opt-in because a step_fn that reads the loss before the optimizer
# (a `loss + reg` term, a NaN guard, a running total, scaler.scale(loss)) would read the previous
# replay's value; bench.py and train_epoch read it only after the step.
_BUMP_DEFER = [None]  # the active deferred_seed_bumps context (or None)
_PENDING_BUMP = {}
_PENDING_LOSS = {}  # device -> (partials workspace, nblk, inv_denom, loss tensor)


class deferred_seed_bumps:
    """Context of a step capture whose dropout counter bumps (and, with ``defer_loss``, the fused
    CE's loss sum) run at the step's end.  ``held``: the CE partials workspaces a deferred loss
    reads at the step's end — the capturing CapturedStep keeps them for the graph's lifetime, so
    no later allocation from the graph's pool can take them over (whichever launch finishes the
    loss: ClipAdam's or the gnn_masked_ce_finish flush_seed_bumps records)."""

    def __init__(self, defer_loss: bool = False):
        self.defer_loss = bool(defer_loss)
        self.held = []

    def __enter__(self):
        _BUMP_DEFER[0] = self
        return self

    def __exit__(self, *exc):
        _BUMP_DEFER[0] = None
        _PENDING_BUMP.clear()
        _PENDING_LOSS.clear()
        return False


def _deferring() -> bool:
    return _BUMP_DEFER[0] is not None and torch.cuda.is_current_stream_capturing()


def defer_loss_sum(device: torch.device, ws: torch.Tensor, nblk: int, inv_denom: float, loss: torch.Tensor) -> bool:
    """Called by the fused CE: True when its loss scalar is left to the step's end (then the CE
    launched with loss = NULL and ``ws`` holds its partials until then)."""
    if not _deferring() or not _BUMP_DEFER[0].defer_loss or device in _PENDING_LOSS:
        return False
    _PENDING_LOSS[device] = (ws, int(nblk), float(inv_denom), loss)
    _BUMP_DEFER[0].held.append(ws)
    return True


def take_loss_sum(device: torch.device):
    """The deferred CE loss of this step ((ws, nblk, inv_denom, loss) — the optimizer's launch
    finishes it), or None."""
    if not _deferring():
        return None
    return _PENDING_LOSS.pop(device, None)


def take_seed_bump(device: torch.device):
    """The counter whose bump this step still owes (the optimizer's launch performs it), or None."""
    if not _deferring():
        return None
    return _PENDING_BUMP.pop(device, None)


def flush_seed_bumps() -> None:
    """Record the owed end-of-step work (a counter add, a loss sum) into the capture in progress."""
    for ctr in _PENDING_BUMP.values():
        ctr.add_(1)
    _PENDING_BUMP.clear()
    for dev, (ws, nblk, inv_denom, loss) in _PENDING_LOSS.items():
        _lib.call("gnn_masked_ce_finish", ws.data_ptr(), nblk, inv_denom, loss.data_ptr(), _lib.stream_handle(dev))
    _PENDING_LOSS.clear()


def dropout_seeds(L: int, p: float, x: torch.Tensor):
    """(per-layer seeds, device counter or None) for the counter-hash dropout of one forward:
    L seeds from torch's CPU generator when eager; per-layer salts plus the device counter,
    bumped once per forward, under HIP-graph capture (see _graph_seed_counter)."""
    if p > 0 and torch.cuda.is_current_stream_capturing():
        ctr = _graph_seed_counter(x.device)
        if _BUMP_DEFER[0] is not None:
            if x.device in _PENDING_BUMP:  # a second forward in the step: its own counter value
                ctr.add_(1)
            _PENDING_BUMP[x.device] = ctr
        else:
            ctr.add_(1)
        return [l + 1 for l in range(L)], ctr
    if p > 0:
        if x.is_cuda:
            _graph_seed_counter(x.device)  # create it outside any capture (a fill inside would replay)
        return torch.randint(0, 2 ** 62, (L,), dtype=torch.int64).tolist(), None
    return [0] * L, None


def tie_output_weights(conv) -> None:
    """Lay the output conv's lin_l.weight and lin_r.weight out as the two halves of ONE [2C, F]
    buffer, which then IS the stacked [W_l ; W_r] the NT epilogue's projection and the TN read
    (no per-step torch.cat).  Called by SAGENet at construction and after every ``_apply``
    (.to() / .cuda() / .float() ...), never from a forward: the Parameter objects, their values,
    optimizer state and state_dict keys are untouched (load_state_dict copies in place and keeps
    the tie; deepcopy keeps it too)."""
    wl, wr = conv.lin_l.weight, conv.lin_r.weight
    if (wl.shape != wr.shape or wl.device != wr.device or wl.dtype != wr.dtype or not wl.is_floating_point()
            or (wl.is_cuda and torch.cuda.is_current_stream_capturing())):
        return
    if _tied_buffer(conv) is not None:
        return
    C = wl.size(0)
    with torch.no_grad():
        buf = torch.cat([wl.detach(), wr.detach()], dim=0).contiguous()
        wl.data = buf[:C]
        wr.data = buf[C:]


def _tied_buffer(conv):
    """The [2C, F] tensor both output weights view (the tie of tie_output_weights), or None."""
    return _tied_buffer_of(conv.lin_l.weight, conv.lin_r.weight)


def _tied_buffer_of(wl, wr):
    """[wl ; wr] as one [2C, F] tensor when wr directly follows wl in one storage, else None."""
    C = wl.size(0)
    if (wl.shape != wr.shape or not wl.is_contiguous() or not wr.is_contiguous() or wl.device != wr.device
            or wl.dtype != wr.dtype or wl.untyped_storage().data_ptr() != wr.untyped_storage().data_ptr()
            or wr.data_ptr() != wl.data_ptr() + wl.numel() * wl.element_size()):
        return None
    return torch.as_strided(wl.detach(), (2 * C, wl.size(1)), (wl.size(1), 1))


def _output_weights(conv):
    """[W_l ; W_r] of the output conv as ONE tensor: the tied buffer (tie_output_weights) when the
    two weights are its halves, else a copy (torch.cat: e.g. after a Parameter was replaced)."""
    buf = _tied_buffer(conv)
    if buf is not None:
        return buf
    return torch.cat([conv.lin_l.weight, conv.lin_r.weight], dim=0).contiguous()


def sage_forward(model, x: torch.Tensor, edge_index: torch.Tensor) -> torch.Tensor:
    plan = get_plan(edge_index, x.size(0), _lib.LOOPS_KEEP)
    L = len(model.convs)
    p = float(model.dropout) if model.training else 0.0
    seeds, ctr = dropout_seeds(L, p, x)
    params = []
    for c in model.convs:
        params += [c.lin_l.weight, c.lin_l.bias, c.lin_r.weight]
    return _FusedSAGE.apply(x, plan, p, seeds, ctr, _output_weights(model.convs[-1]), *params)


# --------------------------------------------------------------------------- SAGEResBNNet layer tail
@functools.lru_cache(maxsize=64)
def _bn_ws_bytes(C: int) -> int:
    nb = _lib.c_size(0)
    _lib.call("gnn_bn_workspace_size", C, nb)
    return int(nb.value)


def _bn_group(bn):
    """torch.distributed when ``bn`` is a SyncBatchNorm1d of an initialised process group, else None."""
    d = getattr(bn, "dist", None)
    return d if (d is not None and d.is_initialized()) else None


class _BNActRes(torch.autograd.Function):
    """h = dropout(relu(BatchNorm1d(z))) + r, training mode (src/models/gnn.py:182-194), on K12
    (csrc/bn.hip): batch statistics in float64 with the nn.BatchNorm1d running-stat update
    (SyncBN: one all-reduce of [Σz | Σz² | n] forward, one of [Σdy | Σdy·x̂] backward), the
    counter-hash dropout of the fused SAGE path, and the whole backward in two passes over z."""

    @staticmethod
    def forward(ctx, z, r, weight, bias, bn, p: float, seed: int, seed_ctr, group):
        z = z.contiguous()
        N, C = z.shape
        dev = z.device
        st = _lib.stream_handle(dev)
        stats = torch.empty(2 * C + 1, dtype=torch.float64, device=dev)
        mean = torch.empty(C, dtype=torch.float32, device=dev)
        invstd = torch.empty(C, dtype=torch.float32, device=dev)
        ws = torch.empty(max(_bn_ws_bytes(C) // 4, 1), dtype=torch.float32, device=dev)
        track = bn.track_running_stats and bn.running_mean is not None
        rm = _lib.ptr(bn.running_mean) if track else None
        rv = _lib.ptr(bn.running_var) if track else None
        nbt = _lib.ptr(bn.num_batches_tracked) if track else None
        mom = -1.0 if bn.momentum is None else float(bn.momentum)
        eps = float(bn.eps)
        _lib.call("gnn_bn_stats_f32", z.data_ptr(), C, N, C, stats.data_ptr(), int(group is None), eps, mom,
                  mean.data_ptr(), invstd.data_ptr(), rm, rv, nbt, ws.data_ptr(), ws.numel() * 4, st)
        if group is not None:
            group.all_reduce(stats)
            _lib.call("gnn_bn_finalize_f32", stats.data_ptr(), C, eps, mom, mean.data_ptr(), invstd.data_ptr(),
                      rm, rv, nbt, st)
        h = torch.empty_like(z)
        if r is not None:
            r = r.contiguous()
        _lib.call("gnn_bn_act_res_fwd_f32", z.data_ptr(), C, _lib.ptr(r), C, N, C, mean.data_ptr(),
                  invstd.data_ptr(), weight.data_ptr(), bias.data_ptr(), float(p), int(seed) & 0xFFFFFFFFFFFFFFFF,
                  _lib.ptr(seed_ctr), h.data_ptr(), C, st)
        ctx.save_for_backward(z, mean, invstd, weight, bias, stats)
        ctx.meta = (float(p), int(seed), seed_ctr, group, r is not None)
        return h

    @staticmethod
    def backward(ctx, dh):
        z, mean, invstd, weight, bias, stats = ctx.saved_tensors
        p, seed, seed_ctr, group, has_r = ctx.meta
        dh = dh.contiguous()
        N, C = z.shape
        dev = z.device
        st = _lib.stream_handle(dev)
        sums = torch.empty(2 * C, dtype=torch.float32, device=dev)
        ws = torch.empty(max(_bn_ws_bytes(C) // 4, 1), dtype=torch.float32, device=dev)
        args = (mean.data_ptr(), invstd.data_ptr(), weight.data_ptr(), bias.data_ptr(), p,
                seed & 0xFFFFFFFFFFFFFFFF, _lib.ptr(seed_ctr))
        _lib.call("gnn_bn_act_bwd_reduce_f32", dh.data_ptr(), C, z.data_ptr(), C, N, C, *args, sums.data_ptr(),
                  ws.data_ptr(), ws.numel() * 4, st)
        local = sums
        if group is not None:  # parameter grads are LOCAL sums (the gradient all-reduce adds the rest)
            local = sums.clone()
            group.all_reduce(sums)
        # dz is written as the right half of an [N, 2C] buffer (tagged): a transform-first SAGEConv
        # below assembles its GEMM gradient [meanᵀ(dz) | dz] in that buffer without a copy
        zbuf = torch.empty((N, 2 * C), dtype=torch.float32, device=dev)
        dz = zbuf[:, C:]
        nb = ctypes.c_int32(0)
        if _BN_COLSUM and N > 0:
            _lib.call("gnn_bn_act_bwd_colsum_blocks", N, C, ctypes.byref(nb))
        if nb.value > 0:  # dz's block column sums too: the bias gradient of the conv below (colsum_of)
            cs = torch.empty(nb.value * C, dtype=torch.float32, device=dev)
            _lib.call("gnn_bn_act_bwd_colsum_f32", dh.data_ptr(), C, z.data_ptr(), C, N, C, *args, sums.data_ptr(),
                      stats[2 * C:].data_ptr(), dz.data_ptr(), 2 * C, cs.data_ptr(), st)
            dz._gnnmp_colsum = cs
        else:
            _lib.call("gnn_bn_act_bwd_f32", dh.data_ptr(), C, z.data_ptr(), C, N, C, *args, sums.data_ptr(),
                      stats[2 * C:].data_ptr(), dz.data_ptr(), 2 * C, st)
        dz._gnnmp_dz = zbuf
        return dz, (dh if has_r else None), local[C:], local[:C], None, None, None, None, None


def bn_fusable(bn) -> bool:
    """nn.BatchNorm1d (or SyncBatchNorm1d) with affine parameters, float32, in training mode."""
    return (isinstance(bn, torch.nn.BatchNorm1d) and bn.training and bn.affine and bn.weight is not None
            and bn.weight.dtype == torch.float32 and bn.weight.is_cuda)


def bn_relu_dropout_residual(z: torch.Tensor, r, bn, p: float, seed: int, seed_ctr) -> torch.Tensor:
    """dropout(relu(bn(z)), p) + r on K12 (training-mode BatchNorm1d / SyncBatchNorm1d)."""
    if z.dtype != torch.float32:
        z = z.float()
    return _BNActRes.apply(z, r, bn.weight, bn.bias, bn, float(p), seed, seed_ctr, _bn_group(bn))


def time_inject_sin(x: torch.Tensor, t_idx: torch.Tensor, dim: int, max_timestep: int) -> torch.Tensor:
    """K13: ``torch.cat([x, sinusoid(t_idx)], 1)`` of SAGEResBNNet (src/models/gnn.py:145-160,
    172-176) in one pass; x float32 [N, F] with unit column stride, no gradient.

    For a registered constant input x (planes.register_input: the training loop's node features)
    the result is a pure function of constants — x and the per-node timesteps — so it is cached on
    x like the graph plan, keyed on (x, t_idx) data pointers and versions, and registered itself:
    later forwards skip the pass, and layer 1's GEMMs (conv and residual projection, both over
    this tensor) read its cached split image instead of splitting it in-kernel every step."""
    key = None
    if is_registered(x):
        key = (x.data_ptr(), x._version, tuple(x.shape), t_idx.data_ptr(), t_idx._version, int(dim),
               int(max_timestep))
        hit = getattr(x, "_gnnmp_time_inject", None)
        if hit is not None and hit[0] == key:
            return hit[1]
    out = _time_inject_sin(x, t_idx, dim, max_timestep)
    if key is not None:
        register_input(out)
        try:
            x._gnnmp_time_inject = (key, out)
        except (AttributeError, RuntimeError):
            pass
    return out


def _time_inject_sin(x: torch.Tensor, t_idx: torch.Tensor, dim: int, max_timestep: int) -> torch.Tensor:
    if x.dim() != 2 or x.stride(1) != 1 or x.dtype != torch.float32:
        x = x.float().contiguous()
    N, Fin = x.shape
    t = t_idx.reshape(-1)
    if t.dtype != torch.int64 or t.stride(0) != 1:
        t = t.to(torch.int64).contiguous()
    if t.numel() != N:
        raise ValueError(f"t_idx has {t.numel()} entries for {N} rows")
    out = torch.empty((N, Fin + dim), dtype=torch.float32, device=x.device)
    _lib.call("gnn_time_inject_sin_f32", x.data_ptr(), _ld(x), N, Fin, t.data_ptr(), int(dim), int(max_timestep),
              out.data_ptr(), _ld(out), _lib.stream_handle(x.device))
    return out
