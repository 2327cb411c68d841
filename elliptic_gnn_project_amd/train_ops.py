"""Fused step ops around the hot path: masked weighted cross entropy and clip + Adam.

``masked_cross_entropy`` is the loss of ``_make_loss_fn`` (src/train_gnn.py:136-183) in its
default configuration — ``F.cross_entropy(logits[train_mask], y[train_mask], weight=cw,
reduction='none').mean()`` (:159-175) — computed over the full logits with the row mask applied
inside one kernel that also writes d(loss)/d(logits) (gnn_masked_ce_f32).  ``ClipAdam`` is
``clip_grad_norm_(params, max_norm)`` (:203-205) followed by ``torch.optim.Adam.step()`` (:206)
in two launches over every parameter (gnn_clip_adam_f32), graph-replay safe (device step count).
Both run on the GPU only; the CPU path keeps the ATen ops.
"""
from __future__ import annotations

import functools
import os
from typing import Iterable

import torch

from . import _lib


def _ws(nbytes: int, device) -> torch.Tensor:
    return torch.empty(max(nbytes // 4, 1), dtype=torch.float32, device=device)


@functools.lru_cache(maxsize=64)
def _ce_ws_bytes(N: int) -> int:
    nb = _lib.c_size(0)
    _lib.call("gnn_masked_ce_workspace_size", N, nb)
    return int(nb.value)


_ONES = {}


def unit_gradient(device) -> torch.Tensor:
    """A persistent scalar 1.0 for ``loss.backward(unit_gradient(dev))``: no per-step fill kernel for
    the implicit gradient, and the fused CE below returns its dlogits without the ``* g`` pass."""
    t = _ONES.get(device)
    if t is None:
        t = torch.ones((), dtype=torch.float32, device=device)
        _ONES[device] = t
    return t


# the masked CE also writes its blocks' column sums of dlogits (gnn_masked_ce_colsum_f32): the
# output layer's bias gradient without a pass over dlogits (GCN / GAT / SAGE-ResBN);
# GNNMP_CE_COLSUM=0: A/B
_CE_COLSUM = os.environ.get("GNNMP_CE_COLSUM", "1") != "0"


class _MaskedCE(torch.autograd.Function):
    """dlogits is written into the right half of an [N, 2C] buffer (``dl._gnnmp_dz``): the fused
    SAGE backward needs dz = [meanᵀ(dlogits) | dlogits] and fills only the left half (no copy)."""

    @staticmethod
    def forward(ctx, logits, y, mask_u8, class_w, inv_denom: float):
        logits = logits.contiguous()
        N, C = logits.shape
        buf = torch.empty((N, 2 * C), dtype=logits.dtype, device=logits.device)
        dl = buf[:, C:]
        loss = torch.empty((), dtype=torch.float32, device=logits.device)
        ws = _ws(_ce_ws_bytes(N), logits.device)
        from .fused import defer_loss_sum

        nblk = max(1, -(-N // 256))  # gnn_masked_ce_f32's partials (256-row blocks)
        deferred = defer_loss_sum(logits.device, ws, nblk, float(inv_denom), loss)  # captured step: at its end
        args = (N, C, logits.data_ptr(), C, y.data_ptr(), mask_u8.data_ptr(), class_w.data_ptr(), float(inv_denom),
                dl.data_ptr(), 2 * C, None if deferred else loss.data_ptr(), ws.data_ptr(), ws.numel() * 4)
        ctx.colsum = None
        if N > 0 and _CE_COLSUM:  # the blocks' column sums of dlogits too: the output layer's bias gradient (colsum_of)
            ctx.colsum = torch.empty(nblk * C, dtype=torch.float32, device=logits.device)
            _lib.call("gnn_masked_ce_colsum_f32", *args, ctx.colsum.data_ptr(), _lib.stream_handle(logits.device))
        else:
            _lib.call("gnn_masked_ce_f32", *args, _lib.stream_handle(logits.device))
        ctx.save_for_backward(buf)
        ctx.C = C
        return loss

    @staticmethod
    def backward(ctx, g):
        (buf,) = ctx.saved_tensors
        dl = buf[:, ctx.C:]
        ones = _ONES.get(g.device)
        if ones is not None and g.data_ptr() == ones.data_ptr():  # d(loss)/d(loss) = 1: dl as is
            dl._gnnmp_dz = buf
            if ctx.colsum is not None:
                dl._gnnmp_colsum = ctx.colsum
            return dl, None, None, None, None
        return dl * g, None, None, None, None


class _PrecomputedCE(torch.autograd.Function):
    """The masked CE a forward already computed (fused_ce_target: gnn_sage_out_mean_ce_f32 ran it
    in the output layer's aggregation): the loss as is, dlogits from its [N, 2C] buffer — the
    same tensors and tags _MaskedCE produces."""

    @staticmethod
    def forward(ctx, logits, ce):
        _, loss, buf, ws = ce
        ctx.save_for_backward(buf)
        ctx.C = buf.size(1) // 2
        ctx.ws = ws  # the loss partials (a deferred loss reads them at the step's end)
        ctx.u = getattr(buf, "_gnnmp_u", None)  # dlogits / max(deg, 1), written by the same launch
        ctx.colsum = getattr(buf, "_gnnmp_colsum", None)  # dlogits' block column sums (gcn_out_ce)
        return loss

    @staticmethod
    def backward(ctx, g):
        (buf,) = ctx.saved_tensors
        dl = buf[:, ctx.C:]
        ones = _ONES.get(g.device)
        if ones is not None and g.data_ptr() == ones.data_ptr():
            dl._gnnmp_dz = buf
            dl._gnnmp_u = ctx.u
            if ctx.colsum is not None:
                dl._gnnmp_colsum = ctx.colsum
            return dl, None
        return dl * g, None


_CE_TARGET = [None]  # (key, y, mask_u8, class_w, inv_denom) of the active fused_ce_target


def _ce_operands(y, mask, class_w, denom, device):
    m8 = mask.view(torch.uint8) if mask.dtype == torch.bool else mask.to(torch.uint8)
    w = class_w.to(device=device, dtype=torch.float32).contiguous()
    y = y.contiguous()
    m8 = m8.contiguous()
    inv = 1.0 / float(denom)
    return (y.data_ptr(), m8.data_ptr(), w.data_ptr(), inv), y, m8, w, inv


class fused_ce_target:
    """Context of a training forward whose loss will be ``masked_cross_entropy(logits, y, mask,
    class_w, denom)`` with exactly these operands: a forward that can compute it on the way does
    (the fused SAGE output layer's mean runs gnn_sage_out_mean_ce_f32 — the F = 2 aggregation and
    the CE in one launch, bit for bit the two launches' results) and masked_cross_entropy then
    returns that result instead of launching the CE.  Every other consumer of the logits sees the
    same logits; a loss with other operands falls back to its own launch.  ``denom`` must be given
    (no host sync)."""

    def __init__(self, y: torch.Tensor, mask: torch.Tensor, class_w: torch.Tensor, denom: float):
        self.args = (y, mask, class_w, denom)

    def __enter__(self):
        y, mask, class_w, denom = self.args
        if y.is_cuda and float(denom) != 0.0:
            _CE_TARGET[0] = _ce_operands(y, mask, class_w, denom, y.device)
        return self

    def __exit__(self, *exc):
        _CE_TARGET[0] = None
        return False


def ce_target():
    """The active fused_ce_target's (key, y, mask_u8, class_w, inv_denom), or None."""
    return _CE_TARGET[0]


def sage_out_mean_ce(plan, z: torch.Tensor, C: int, bias, target, colsum: bool = False):
    """logits = mean_{j->i} z[j, :C] + z[i, C:] + bias and the target's masked CE in one launch
    (include/gnnmp.h gnn_sage_out_mean_ce_f32).  Returns (logits, ce) — ce for _PrecomputedCE.
    ``colsum``: also dlogits' block column sums (the output bias gradient, aggregation.colsum_of)."""
    from .fused import defer_loss_sum

    key, y, m8, w, inv = target
    N, dev = z.size(0), z.device
    logits = torch.empty((N, C), dtype=torch.float32, device=dev)
    buf = torch.empty((N, 2 * C), dtype=torch.float32, device=dev)
    u = torch.empty((N, C), dtype=torch.float32, device=dev)  # dlogits / max(deg, 1): meanᵀ as a plain sum
    loss = torch.empty((), dtype=torch.float32, device=dev)
    ws = _ws(_ce_ws_bytes(N), dev)
    nblk = max(1, -(-N // 256))
    deferred = defer_loss_sum(dev, ws, nblk, inv, loss)  # captured step with defer_loss: at its end
    cs = torch.empty(nblk * C, dtype=torch.float32, device=dev) if (colsum and _CE_COLSUM) else None
    _lib.call("gnn_sage_out_mean_ce_f32", plan.c_graph, plan.deg.data_ptr(), z.data_ptr(), int(z.stride(0)), int(C),
              _lib.ptr(bias), logits.data_ptr(), C, y.data_ptr(), m8.data_ptr(), w.data_ptr(), float(inv),
              buf.data_ptr() + C * 4, 2 * C, u.data_ptr(), C, _lib.ptr(cs), None if deferred else loss.data_ptr(),
              ws.data_ptr(), ws.numel() * 4, _lib.stream_handle(dev))
    buf._gnnmp_u = u
    if cs is not None:
        buf._gnnmp_colsum = cs
    return logits, (key, loss, buf, ws)


def gcn_out_ce(plan, t: torch.Tensor, bias, target):
    """logits = Â·t + bias (GCN's output aggregation over a LOOPS_REPLACE plan, C <= 2) and the
    target's masked CE in one launch (include/gnnmp.h gnn_gcn_out_ce_f32), dlogits' block column
    sums beside them (the output bias gradient, aggregation.colsum_of).  Returns (logits, ce) — ce
    for _PrecomputedCE."""
    from .fused import defer_loss_sum

    key, y, m8, w, inv = target
    N, C, dev = t.size(0), t.size(1), t.device
    logits = torch.empty((N, C), dtype=torch.float32, device=dev)
    buf = torch.empty((N, 2 * C), dtype=torch.float32, device=dev)
    loss = torch.empty((), dtype=torch.float32, device=dev)
    ws = _ws(_ce_ws_bytes(N), dev)
    nblk = max(1, -(-N // 256))
    cs = torch.empty(nblk * C, dtype=torch.float32, device=dev) if _CE_COLSUM else None
    deferred = defer_loss_sum(dev, ws, nblk, inv, loss)
    _lib.call("gnn_gcn_out_ce_f32", plan.c_graph, plan.dinv.data_ptr(), t.data_ptr(), int(t.stride(0)), int(C),
              _lib.ptr(bias), logits.data_ptr(), C, y.data_ptr(), m8.data_ptr(), w.data_ptr(), float(inv),
              buf.data_ptr() + C * 4, 2 * C, _lib.ptr(cs), None if deferred else loss.data_ptr(), ws.data_ptr(),
              ws.numel() * 4, _lib.stream_handle(dev))
    if cs is not None:
        buf._gnnmp_colsum = cs
    return logits, (key, loss, buf, ws)


def gat_out(plan, p, target=None):
    """GATNet's output conv (heads 1, C <= 2, no concat / act / dropout) in the narrow form
    (include/gnnmp.h gnn_gat_out_ce_f32), ``p`` the GnnGatFwdParams of the call; with ``target`` the
    masked CE in the same launch, dlogits' block column sums beside them.  Returns ce (for
    _PrecomputedCE) or None."""
    from .fused import defer_loss_sum

    N, C = plan.num_nodes, int(p.chans)
    dev = plan.device
    if target is None:
        _lib.call("gnn_gat_out_ce_f32", plan.c_graph, p, None, None, None, 0.0, None, 0, None, None, None, 0,
                  _lib.stream_handle(dev))
        return None
    key, y, m8, w, inv = target
    buf = torch.empty((N, 2 * C), dtype=torch.float32, device=dev)
    loss = torch.empty((), dtype=torch.float32, device=dev)
    ws = _ws(_ce_ws_bytes(N), dev)
    nblk = max(1, -(-N // 256))
    cs = torch.empty(nblk * C, dtype=torch.float32, device=dev) if _CE_COLSUM else None
    deferred = defer_loss_sum(dev, ws, nblk, inv, loss)
    _lib.call("gnn_gat_out_ce_f32", plan.c_graph, p, y.data_ptr(), m8.data_ptr(), w.data_ptr(), float(inv),
              buf.data_ptr() + C * 4, 2 * C, _lib.ptr(cs), None if deferred else loss.data_ptr(), ws.data_ptr(),
              ws.numel() * 4, _lib.stream_handle(dev))
    if cs is not None:
        buf._gnnmp_colsum = cs
    return (key, loss, buf, ws)


def masked_cross_entropy(logits: torch.Tensor, y: torch.Tensor, mask: torch.Tensor, class_w: torch.Tensor,
                         denom: float | None = None) -> torch.Tensor:
    """Σ_{i: mask_i} CE_w(logits_i, y_i) / denom (denom defaults to mask.sum(): the reference's .mean()).

    ``mask`` is a bool/uint8 [N] tensor, ``y`` int64 [N] (labels of unmasked rows are ignored).
    """
    if not logits.is_cuda:
        raise RuntimeError("masked_cross_entropy runs on the GPU (libgnnmp); use the ATen loss on CPU")
    if logits.dtype != torch.float32:
        logits = logits.float()
    if denom is None:
        denom = float(mask.sum())  # host sync; pass denom to avoid it
    if float(denom) == 0.0:
        # empty selection: the reference's loss_vec.mean() is NaN and its gradient is zero
        return logits.sum() * 0.0 + float("nan")
    key, y, m8, w, inv = _ce_operands(y, mask, class_w, denom, logits.device)  # bool mask: no copy
    ce = getattr(logits, "_gnnmp_ce", None)
    if ce is not None and ce[0] == key:  # the forward already computed it (fused_ce_target)
        return _PrecomputedCE.apply(logits, ce)
    return _MaskedCE.apply(logits, y, m8, w, inv)


# Σg² folded into the gradients' producer (ABI 20).  A ClipAdam registers (partials buffer, step
# counter) per device; a backward whose ONE weight-gradient TN writes every gradient of the model
# (the fused 2-layer SAGE) passes them to that TN, whose ordered reduce then also writes the norm
# partials and the step snapshot, and records what it wrote; the next ClipAdam.step takes the
# record when its gradients are exactly views of that output — then its launch pair is one launch.
_GRAD_SQ_REQ: dict = {}   # device -> (partials buffer, step tensor)
_GRAD_SQ_DONE: dict = {}  # device -> (out, n_out, (skip_lo, skip_hi), nb, partials buffer, step tensor, out._version)
_GRAD_SQ_CAP = 2048       # >= 2 nb + 1 for every TN output (Nr <= 128, K <= 384: nb <= 779)


def grad_sq_request(device):
    """(partials buffer, step tensor) of the ClipAdam on ``device`` that takes Σg² from the producer."""
    return _GRAD_SQ_REQ.get(device)


def grad_sq_produced(device, rec) -> None:
    """Record (or clear, rec None) the norm partials this step's gradient producer wrote."""
    if rec is None:
        _GRAD_SQ_DONE.pop(device, None)
    else:
        _GRAD_SQ_DONE[device] = rec


def _tiles(rec, ps) -> bool:
    """The grads of ``ps`` are views of rec's out that tile [0, n_out) minus the skipped range, and
    nothing wrote them in place since the producer recorded its Σg² (the version counter views share)."""
    out, n_out, (lo, hi) = rec[0], rec[1], rec[2]
    if out._version != rec[6]:
        return False
    base, sto, spans = out.data_ptr(), out.untyped_storage().data_ptr(), []
    for p in ps:
        g = p.grad  # (AccumulateGrad adopts the backward's views detached: same storage, no _base)
        if (g is None or g.untyped_storage().data_ptr() != sto or not g.is_contiguous()
                or g.dtype != torch.float32):
            return False
        off = (g.data_ptr() - base) // 4
        spans.append((off, off + g.numel()))
    pos = 0
    for a, b in sorted(spans):
        if pos == lo:
            pos = hi
        if a != pos:
            return False
        pos = b
    if pos == lo:
        pos = hi
    return pos == n_out


class ClipAdam(torch.optim.Optimizer):
    """``clip_grad_norm_(max_norm)`` + ``Adam`` (L2 weight decay, amsgrad off) in two kernels.

    Same update as ``torch.optim.Adam(lr, betas, eps, weight_decay)`` preceded by
    ``torch.nn.utils.clip_grad_norm_(params, max_norm)`` (grads scaled in place by
    min(1, max_norm / (‖g‖ + 1e-6))); ``max_norm=None`` skips clipping.  The step counter lives on
    the device, so a captured HIP graph replays it.  ``last_norm`` holds the pre-clip total norm.
    """

    def __init__(self, params: Iterable, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 max_norm: float | None = 1.0, skip_nonfinite: bool = False):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        # skip_nonfinite: GradScaler.step's skip of an update whose gradients hold inf / NaN (the
        # AMP configurations, src/train_gnn.py:202-207; train_gnn.train_epoch)
        self.skip_nonfinite = bool(skip_nonfinite)
        if max_norm and len(self.param_groups) > 1:
            raise ValueError("ClipAdam clips over one parameter group (as clip_grad_norm_ over model.parameters())")
        self.max_norm = max_norm
        self._ws = None
        self._sq = None  # norm partials written by the gradients' producer (grad_sq_request)
        self.last_folded = False  # the last step took them (one launch instead of two)
        self._groups = {}
        self.last_norm = None

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for gi, group in enumerate(self.param_groups):
            ps = [p for p in group["params"] if p.grad is not None]
            if not ps:
                continue
            dev = ps[0].device
            if self._ws is None:
                if not ps[0].is_cuda:
                    raise RuntimeError("ClipAdam runs on the GPU (libgnnmp)")
                nb = _lib.c_size(0)
                _lib.call("gnn_clip_adam_workspace_size", nb)
                self._ws = torch.zeros(max(int(nb.value) // 4, 1), dtype=torch.float32, device=dev)  # (its counter word starts at 0)
                self.last_norm = torch.zeros(1, dtype=torch.float32, device=dev)
            if "step_t" not in group:  # device step counter of this group (advanced by the kernel)
                group["step_t"] = torch.zeros(1, dtype=torch.float32, device=dev)
            # the ctypes argument block is rebuilt only when a pointer or a hyper-parameter changed
            # (the caching allocator usually hands every step's grads the same addresses)
            key = (tuple(p.grad.data_ptr() for p in ps), tuple(p.data_ptr() for p in ps), group["lr"],
                   group["betas"], group["eps"], group["weight_decay"], self.max_norm, self.skip_nonfinite)
            cached = self._groups.get(gi)
            if cached is None or cached[0] != key:
                cached = (key, self._build(group, ps))
                self._groups[gi] = cached
            from .fused import take_loss_sum, take_seed_bump

            # a captured step's end-of-step work rides in this launch: the dropout counter's bump and
            # the fused CE's loss sum
            g = cached[1]
            bump = take_seed_bump(dev)
            g.bump_counter = bump.data_ptr() if bump is not None else None
            ls = take_loss_sum(dev) if gi == 0 else None
            if ls is not None:
                g.loss_partial, g.loss_nblk, g.loss_scale, g.loss_out = ls[0].data_ptr(), ls[1], ls[2], ls[3].data_ptr()
            rec = _GRAD_SQ_DONE.pop(dev, None) if gi == 0 else None
            self.last_folded = (rec is not None and len(self.param_groups) == 1 and rec[5] is group["step_t"]
                                and _tiles(rec, ps))
            if self.last_folded:  # one launch: Σg² came with the gradients
                g.grad_sq_partial, g.grad_sq_nblk = rec[4].data_ptr(), rec[3]
            _lib.call("gnn_clip_adam_f32", g, group["step_t"].data_ptr(), self.last_norm.data_ptr(),
                      self._ws.data_ptr(), self._ws.numel() * 4, _lib.stream_handle(dev))
            g.bump_counter = g.loss_partial = g.loss_out = g.grad_sq_partial = None
            g.loss_nblk, g.loss_scale, g.grad_sq_nblk = 0, 0.0, 0  # (the partials workspace is held by the capturing CapturedStep)
            if len(self.param_groups) == 1:  # the next backward's producer may fold Σg²
                if self._sq is None:
                    self._sq = torch.zeros(_GRAD_SQ_CAP, dtype=torch.float32, device=dev)
                _GRAD_SQ_REQ[dev] = (self._sq, group["step_t"])
        return loss

    @staticmethod
    def supports(params) -> bool:
        """True when one ClipAdam launch pair covers ``params`` (≤ ADAM_MAX_TENSORS fp32 tensors);
        make_optimizer falls back to torch.optim.Adam + clip_grad_norm_ otherwise."""
        ps = list(params)
        return 0 < len(ps) <= _lib.ADAM_MAX_TENSORS and all(p.dtype == torch.float32 for p in ps)

    def _build(self, group, ps):
        if len(ps) > _lib.ADAM_MAX_TENSORS:
            raise ValueError(f"ClipAdam: at most {_lib.ADAM_MAX_TENSORS} tensors per group "
                             "(use torch.optim.Adam + clip_grad_norm_; make_optimizer does so)")
        grp = _lib.GnnAdamGroup()
        grp.num_tensors = len(ps)
        grp.lr, (grp.beta1, grp.beta2) = group["lr"], group["betas"]
        grp.eps, grp.weight_decay = group["eps"], group["weight_decay"]
        grp.max_norm = float(self.max_norm) if self.max_norm else 0.0
        grp.skip_nonfinite = int(self.skip_nonfinite)
        for j, p in enumerate(ps):
            st = self.state[p]
            if not st:
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                st["step"] = group["step_t"]
            if not (p.is_contiguous() and p.grad.is_contiguous() and p.dtype == torch.float32):
                raise ValueError("ClipAdam needs contiguous fp32 params and grads")
            t = grp.tensors[j]
            t.param, t.grad = p.data_ptr(), p.grad.data_ptr()
            t.exp_avg, t.exp_avg_sq = st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr()
            t.numel = p.numel()
        return grp
