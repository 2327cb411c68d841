"""The four GNN families of the reference (src/models/gnn.py), on libgnnmp convs.

Same constructor signatures, ``forward(x, edge_index, t_idx=None)``, attribute names
(``convs``, ``bns``, ``res_projs``, ``time_emb``, ``time_embed_dim``) and hence the same
``state_dict`` keys as the reference, so ``best.ckpt`` files and the reference's
train/eval callers (src/train_gnn.py:67-104, src/analysis/*) work unchanged.

  GCNNet        gnn.py:14-32   GCNConv stack, ReLU + dropout between layers
  SAGENet       gnn.py:35-53   SAGEConv stack, ReLU + dropout between layers
  GATNet        gnn.py:56-76   GATConv(heads, concat) stack, ELU + dropout; last layer 1 head, mean
  SAGEResBNNet  gnn.py:82-194  time embedding + SAGEConv + BatchNorm + ReLU + dropout + residual
"""
from __future__ import annotations

import math
import os
from typing import Callable, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from . import fused as _fused
from .conv import GATConv, GCNConv, SAGEConv
from .linear import Linear

__all__ = ["GCNNet", "SAGENet", "GATNet", "SAGEResBNNet"]


class _StackedConvNet(nn.Module):
    """conv -> act -> dropout for every layer but the last; the last conv gives logits."""

    act: Callable[[torch.Tensor], torch.Tensor] = staticmethod(F.relu)

    def __init__(self, convs, dropout: float):
        super().__init__()
        if len(convs) < 2:
            raise AssertionError("layers must be >= 2")  # reference: assert layers >= 2
        self.dropout = dropout
        self.convs = nn.ModuleList(convs)

    def forward(self, x: torch.Tensor, edge_index: torch.Tensor, t_idx: Optional[torch.Tensor] = None):
        *hidden, last = self.convs
        h = x
        for conv in hidden:
            h = F.dropout(self.act(conv(h, edge_index)), p=self.dropout, training=self.training)
        return last(h, edge_index)


def _widths(in_dim: int, hidden_dim: int, layers: int, num_classes: int):
    if layers < 2:
        raise AssertionError("layers must be >= 2")
    ins = [in_dim] + [hidden_dim] * (layers - 1)
    outs = [hidden_dim] * (layers - 1) + [num_classes]
    return list(zip(ins, outs))


class GCNNet(_StackedConvNet):
    """On the GPU the whole network runs as one fused autograd node (fused.py _FusedGCN): bias,
    ReLU and dropout in the aggregation's store, their backward in the skinny GEMM's epilogue
    (counter-hash dropout, as SAGENet).  ``fused = False`` selects the per-conv path."""

    fused = True

    def __init__(self, in_dim, hidden_dim=128, layers=3, dropout=0.2, num_classes=2):
        super().__init__([GCNConv(a, b) for a, b in _widths(in_dim, hidden_dim, layers, num_classes)], dropout)

    def forward(self, x: torch.Tensor, edge_index: torch.Tensor, t_idx: Optional[torch.Tensor] = None):
        if self.fused and x.is_cuda and _fused.gcn_fusable(self):
            return _fused.gcn_forward(self, x, edge_index)
        return super().forward(x, edge_index, t_idx)


class SAGENet(_StackedConvNet):
    """When the shape allows (narrow 2-class output, widths within the kernels' limits) the whole
    network runs as one fused autograd node (fused.py): aggregate-first SAGE layers on the MFMA
    GEMM with bias/ReLU/dropout and the output layer's transform fused into its epilogue.
    ``fused = False`` selects the per-conv path (same kernels, layer by layer)."""

    fused = True

    def __init__(self, in_dim, hidden_dim=128, layers=3, dropout=0.2, num_classes=2):
        super().__init__([SAGEConv(a, b) for a, b in _widths(in_dim, hidden_dim, layers, num_classes)], dropout)
        _fused.tie_output_weights(self.convs[-1])

    def _apply(self, fn, recurse=True):
        # .to() / .cuda() / .float() give each weight new storage: re-tie the output conv's pair
        # (the fused path reads [W_l ; W_r] as one buffer, fused.tie_output_weights)
        out = super()._apply(fn, recurse)
        _fused.tie_output_weights(self.convs[-1])
        return out

    def __deepcopy__(self, memo):
        import copy

        new = self.__class__.__new__(self.__class__)
        memo[id(self)] = new
        new.__setstate__(copy.deepcopy(self.__dict__, memo))
        _fused.tie_output_weights(new.convs[-1])
        return new

    def forward(self, x: torch.Tensor, edge_index: torch.Tensor, t_idx: Optional[torch.Tensor] = None):
        if self.fused and x.is_cuda and _fused.fusable(self):
            return _fused.sage_forward(self, x, edge_index)
        return super().forward(x, edge_index, t_idx)


class GATNet(_StackedConvNet):
    """The hidden layers' ``dropout(elu(conv(h)))`` (gnn.py:72-74) runs on the attention kernel's
    store (ELU, then the same counter-hash dropout as the fused SAGE path, oracle/dropout_hash.py);
    explain mode falls back to F.elu / F.dropout around each conv."""

    act = staticmethod(F.elu)

    def __init__(self, in_dim, hidden_dim=128, layers=3, dropout=0.2, num_classes=2, heads=4):
        per_head = hidden_dim // heads  # reference: hidden_dim // heads channels per head
        convs = [GATConv(in_dim if i == 0 else hidden_dim, per_head, heads=heads) for i in range(layers - 1)]
        convs.append(GATConv(hidden_dim, num_classes, heads=1, concat=False))
        super().__init__(convs, dropout)

    def forward(self, x: torch.Tensor, edge_index: torch.Tensor, t_idx: Optional[torch.Tensor] = None):
        if not x.is_cuda or any(getattr(c, "explain", False) for c in self.convs):
            return super().forward(x, edge_index, t_idx)
        *hidden, last = self.convs
        p = float(self.dropout) if self.training else 0.0
        seeds, ctr = _fused.dropout_seeds(len(self.convs), p, x)
        h = x
        # the last hidden layer writes the output conv's lin(h) beside its store, and its backward
        # forms dh from d lin(h) in the kernel (ABI 24): h is never read back or its gradient stored
        proj = (_GAT_PROJ and hidden and last.heads == 1 and not last.concat and last.out_channels <= 4
                and (hidden[-1].heads * hidden[-1].out_channels) % 4 == 0)
        for i, conv in enumerate(hidden):
            post = (_lib.ACT_ELU, p, seeds[i], ctr)
            if proj and i == len(hidden) - 1:
                return last._forward_from_xh(conv._forward_proj(h, edge_index, last.lin.weight, post), edge_index)
            h = conv(h, edge_index, _post=post)
        return last(h, edge_index)


_RES_FOLD = os.environ.get("GNNMP_RES_FOLD", "1") != "0"  # A/B: 0 = autograd adds the residual's gradient
_GAT_PROJ = os.environ.get("GNNMP_GAT_PROJ", "1") != "0"  # A/B: 0 = the output conv's lin as its own GEMMs


class SAGEResBNNet(nn.Module):
    """SAGE + BatchNorm + residual, optional timestep embedding concatenated to the input.

    time_embed_type: 'learned' (nn.Embedding(max_timestep, dim)), 'sin' (fixed sin/cos of
    2π·k·(t-1)/(T-1), k = 1..dim/2, zero-padded to dim), anything else / dim 0: none.

    On the GPU in training mode each hidden layer's ``dropout(relu(bn(z))) + res_proj(h)`` runs
    on K12 (fused.bn_relu_dropout_residual: float64 batch statistics, the BatchNorm1d running-stat
    update, SyncBN when the BN is a SyncBatchNorm1d, counter-hash dropout as SAGENet); eval mode
    and CPU keep nn.BatchNorm1d / F.relu / F.dropout.  ``fused_bn = False`` selects that path.
    """

    def __init__(self, in_dim, hidden_dim=128, layers=3, dropout=0.2, num_classes=2, use_bn=True,
                 residual=True, time_embed_dim=0, time_embed_type="learned", max_timestep=50):
        super().__init__()
        if layers < 2:
            raise AssertionError("layers must be >= 2")
        self.dropout = float(dropout)
        self.use_bn = bool(use_bn)
        self.residual = bool(residual)  # kept as an attribute; the reference always adds the residual
        self.time_embed_dim = int(time_embed_dim)
        self.time_embed_type = str(time_embed_type)
        self.max_timestep = int(max_timestep)
        self.time_emb = None
        if self.time_embed_dim > 0 and self.time_embed_type in ("learned", "sin"):
            if self.time_embed_type == "learned":
                self.time_emb = nn.Embedding(self.max_timestep, self.time_embed_dim)
            in_dim = in_dim + self.time_embed_dim
        else:
            self.time_embed_dim, self.time_embed_type = 0, "none"

        dims = _widths(in_dim, hidden_dim, layers, num_classes)
        self.convs = nn.ModuleList(SAGEConv(a, b) for a, b in dims)
        self.bns = nn.ModuleList(nn.BatchNorm1d(hidden_dim) for _ in range(layers - 1)) if self.use_bn \
            else nn.ModuleList()
        self.res_projs = nn.ModuleList(
            nn.Identity() if a == b else Linear(a, b, bias=False) for a, b in dims[:-1]
        )

    def _sinusoid(self, t_idx: torch.Tensor) -> Optional[torch.Tensor]:
        dim = self.time_embed_dim
        if dim <= 0:
            return None
        t = (t_idx.long() - 1).clamp(0, self.max_timestep - 1).to(torch.float32)
        t = t / max(float(self.max_timestep - 1), 1.0)
        half = dim // 2
        freqs = torch.arange(1, half + 1, device=t.device, dtype=t.dtype) * (2.0 * math.pi)
        ang = t[:, None] * freqs[None, :]
        feat = torch.cat([torch.sin(ang), torch.cos(ang)], dim=1)
        if feat.size(1) < dim:
            feat = F.pad(feat, (0, dim - feat.size(1)))
        return feat

    def _inject_time(self, x: torch.Tensor, t_idx: Optional[torch.Tensor]) -> torch.Tensor:
        if self.time_embed_dim <= 0 or t_idx is None:
            return x
        if self.time_embed_type == "learned":
            te = self.time_emb((t_idx.long() - 1).clamp(0, self.max_timestep - 1))
        elif self.time_embed_type == "sin":
            if x.is_cuda and not x.requires_grad and x.dim() == 2:
                return _fused.time_inject_sin(x, t_idx, self.time_embed_dim, self.max_timestep)  # K13
            te = self._sinusoid(t_idx)
        else:
            return x
        return torch.cat([x, te], dim=1)

    fused_bn = True  # training-mode BN + ReLU + dropout + residual on K12 (fused.bn_relu_dropout_residual)

    def forward(self, x: torch.Tensor, edge_index: torch.Tensor, t_idx: Optional[torch.Tensor] = None):
        h = self._inject_time(x, t_idx)
        *hidden, last = self.convs
        fuse = self.fused_bn and self.use_bn and self.training and x.is_cuda
        seeds, ctr = (_fused.dropout_seeds(len(self.convs), self.dropout, h) if fuse else (None, None))
        for li, conv in enumerate(hidden):
            if fuse and _fused.bn_fusable(self.bns[li]):
                if isinstance(self.res_projs[li], nn.Identity) and _RES_FOLD:  # the residual's gradient in conv's dx
                    z, r = conv.forward_with_residual(h, edge_index)
                else:
                    z, r = conv(h, edge_index), self.res_projs[li](h)
                h = _fused.bn_relu_dropout_residual(z, r, self.bns[li], self.dropout, seeds[li], ctr)
                continue
            z = conv(h, edge_index)
            if self.use_bn:
                z = self.bns[li](z)
            z = F.dropout(F.relu(z), p=self.dropout, training=self.training)
            h = z + self.res_projs[li](h)
        return last(h, edge_index)
