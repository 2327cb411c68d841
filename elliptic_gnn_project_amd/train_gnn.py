"""Full-batch training driver — the reference's src/train_gnn.py surface on libgnnmp models.

Kept from the reference (same names, same YAML keys, same semantics):
  build_model         src/train_gnn.py:67-104
  get_device          :107-113   (the HIP device is required: there is no CPU path)
  class_weight        :116-123
  _make_loss_fn       :136-183   (CE with class weights, focal, time weighting, embed L2)
  train_epoch         :187-209   (AMP autocast + GradScaler + clip_grad_norm_ + Adam)
  eval_split          :248-257
  main                :282-564   (masks window, time scalar, symmetrize, early stopping on val
                                  PR-AUC, best-state restore, temperature scaling, metrics.json,
                                  best.ckpt, optional hub ablation)
New optional keys: ``synthetic`` (dict of synthetic_elliptic kwargs, used when no
processed graph exists), ``graph_file`` (PyG-free .npz written by dataset_elliptic.save_graph).
The mini-batch NeighborLoader path (:212-245, :329-348) is not implemented.
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import random
from typing import Dict

import numpy as np
import torch
import torch.nn.functional as F
import yaml

from .dataset_elliptic import GraphData, load_graph, prepare_inputs, synthetic_elliptic
from .gnn import GATNet, GCNNet, SAGENet, SAGEResBNNet


# ----------------------------------------------------------------------------- setup
def set_seed(seed: int = 42) -> None:
    """src/utils/common.py:11-17."""
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    torch.cuda.manual_seed_all(seed)


def build_model(arch: str, in_dim: int, cfg: Dict):
    if arch == "gcn":
        return GCNNet(in_dim, hidden_dim=cfg["hidden_dim"], layers=cfg["layers"], dropout=cfg["dropout"])
    if arch == "sage":
        return SAGENet(in_dim, hidden_dim=cfg["hidden_dim"], layers=cfg["layers"], dropout=cfg["dropout"])
    if arch == "gat":
        return GATNet(in_dim, hidden_dim=cfg["hidden_dim"], layers=cfg["layers"], heads=cfg.get("heads", 4),
                      dropout=cfg["dropout"])
    if arch in ("sage_resbn", "sage_bn", "sage_res"):
        return SAGEResBNNet(
            in_dim,
            hidden_dim=cfg.get("hidden_dim", 128),
            layers=cfg.get("layers", 3),
            dropout=cfg.get("dropout", 0.2),
            num_classes=2,
            use_bn=cfg.get("use_bn", True),
            residual=cfg.get("residual", True),
            time_embed_dim=cfg.get("time_embed_dim", 0),
            time_embed_type=cfg.get("time_embed_type", "learned"),
            max_timestep=cfg.get("max_timestep", 49),
        )
    raise ValueError("Unknown arch")


def get_device(cfg: Dict) -> torch.device:
    forced = cfg.get("device", "auto")
    if forced == "cpu" or not torch.cuda.is_available():
        raise RuntimeError(
            "elliptic_gnn_project_amd trains on the MI355X (HIP) device only; "
            f"device={forced!r}, torch.cuda.is_available()={torch.cuda.is_available()}. "
            "The CPU path of the reference is the PyG-CPU baseline (oracle/pyg_ref.py)."
        )
    return torch.device("cuda", torch.cuda.current_device())


def class_weight(train_y: torch.Tensor) -> torch.Tensor:
    pos = int((train_y == 1).sum().item())
    neg = int((train_y == 0).sum().item())
    if pos == 0 or neg == 0:
        return torch.tensor([1.0, 1.0], dtype=torch.float32)
    return torch.tensor([(pos + neg) / (2.0 * neg), (pos + neg) / (2.0 * pos)], dtype=torch.float32)


def _model_uses_time_embed(model) -> bool:
    return getattr(model, "time_embed_dim", 0) > 0


def _norm_train_time(t_vec, t_min, t_max):
    return (t_vec.float() - float(t_min)) / max(float(t_max - t_min), 1.0)


def _make_loss_fn(cfg: Dict, cw: torch.Tensor, model, t_min: int, t_max: int):
    scheme = str(cfg.get("time_loss_weighting", "none"))
    embed_l2 = float(cfg.get("time_embed_l2", 0.0))
    focal = bool(cfg.get("focal_loss", False))
    gamma = float(cfg.get("focal_gamma", 2.0))
    cw_dev = {}

    def loss_fn(logits, target, t_idx=None, denom=None):
        if focal:
            ce = F.cross_entropy(logits, target, reduction="none")
            pt = torch.softmax(logits, dim=1).gather(1, target.view(-1, 1)).squeeze(1)
            loss_vec = ((1 - pt) ** gamma) * ce
        else:
            w = cw_dev.get(logits.device)
            if w is None:
                w = cw_dev[logits.device] = cw.to(logits.device)
            loss_vec = F.cross_entropy(logits, target, weight=w, reduction="none")
        if scheme != "none" and t_idx is not None:
            wt = _norm_train_time(t_idx, t_min, t_max).to(logits.device)
            if scheme == "sqrt":
                wt = torch.sqrt(torch.clamp(wt, min=0.0))
            elif scheme != "linear":
                raise ValueError(f"unknown time_loss_weighting={scheme}")
            loss_vec = loss_vec * torch.clamp(wt, min=1e-3)
        # ``denom``: global sample count for timestep-partitioned data parallelism, so the
        # sum over ranks equals the single-device .mean() (src/train_gnn.py:175).
        loss = loss_vec.mean() if denom is None else loss_vec.sum() / float(denom)
        if embed_l2 > 0.0 and getattr(model, "time_emb", None) is not None:
            loss = loss + embed_l2 * model.time_emb.weight.pow(2).mean()
        return loss

    def full(logits, y_all, mask, denom=None, t_idx_all=None):
        """The same loss from the full logits and the row mask: on the GPU in the default
        configuration one fused kernel (train_ops.masked_cross_entropy); else loss_fn on the rows."""
        if loss_fn.plain and logits.is_cuda and logits.dtype == torch.float32:
            from .train_ops import masked_cross_entropy
            w = cw_dev.get(logits.device)
            if w is None:
                w = cw_dev[logits.device] = cw.to(logits.device)
            return masked_cross_entropy(logits, y_all, mask, w, denom=denom)
        idx = mask.nonzero().squeeze(1)
        t_sel = t_idx_all.index_select(0, idx) if t_idx_all is not None else None
        return loss_fn(logits.index_select(0, idx), y_all.index_select(0, idx), t_sel, denom=denom)

    loss_fn.plain = not focal and scheme == "none" and embed_l2 == 0.0
    loss_fn.full = full
    return loss_fn


def _autocast(device, enabled: bool):
    return torch.amp.autocast(device_type=device.type, enabled=enabled)


# ----------------------------------------------------------------------------- loops
def _rows(t: torch.Tensor, data, split: str) -> torch.Tensor:
    """t[data.<split>_mask] via the precomputed index when available (no per-step host sync)."""
    idx = getattr(data, f"{split}_idx", None)
    return t.index_select(0, idx) if idx is not None else t[getattr(data, f"{split}_mask")]


def _clips_itself(optimizer) -> bool:
    from .train_ops import ClipAdam
    return isinstance(optimizer, ClipAdam) and bool(optimizer.max_norm)


def make_optimizer(model, cfg: Dict, device, use_amp: bool):
    """Adam(lr, weight_decay) (src/train_gnn.py:357).  On the GPU without AMP: ClipAdam, the
    fused clip_grad_norm_(grad_clip) + Adam step (train_ops.py); otherwise torch.optim.Adam."""
    if device.type == "cuda" and not use_amp:
        from .train_ops import ClipAdam
        clip = cfg.get("grad_clip", 0)
        return ClipAdam(model.parameters(), lr=cfg["lr"], weight_decay=cfg["weight_decay"],
                        max_norm=float(clip) if clip and clip > 0 else None)
    return torch.optim.Adam(model.parameters(), lr=cfg["lr"], weight_decay=cfg["weight_decay"])


def train_epoch(model, data, edge_index, optimizer, loss_fn, scaler, use_amp, cfg, device, sync=True):
    """One full-batch step (src/train_gnn.py:187-209).  ``sync=False`` keeps the loss on device."""
    model.train()
    optimizer.zero_grad(set_to_none=True)
    with _autocast(device, use_amp):
        logits = model(data.x, edge_index, data.timestep if _model_uses_time_embed(model) else None)
        t_idx = _rows(data.timestep, data, "train") if cfg.get("time_loss_weighting", "none") != "none" else None
        if getattr(loss_fn, "plain", False) and logits.is_cuda and not use_amp:
            loss = loss_fn.full(logits, data.y, data.train_mask, denom=getattr(data, "n_train", None))
        else:
            loss = loss_fn(_rows(logits, data, "train"), _rows(data.y, data, "train"), t_idx)
    scaler.scale(loss).backward()
    if cfg.get("grad_clip", 0) and cfg["grad_clip"] > 0 and not _clips_itself(optimizer):
        scaler.unscale_(optimizer)
        torch.nn.utils.clip_grad_norm_(model.parameters(), cfg["grad_clip"])
    scaler.step(optimizer)
    scaler.update()
    optimizer.zero_grad(set_to_none=True)
    return float(loss.item()) if sync else loss.detach()


class CapturedStep:
    """A training step captured once into a HIP graph and replayed (torch.cuda.CUDAGraph).

    ``step_fn`` must be capture-safe: static input tensors, no host syncs, optimizer built
    with ``capturable=True``.  The fused SAGE path switches its dropout seed to a device
    counter under capture, so every replay draws a new mask.  Replaying removes the host's
    per-kernel launch cost (≈40 launches per step) and the gaps between kernels.
    """

    def __init__(self, step_fn, warmup: int = 3):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                step_fn()
        torch.cuda.current_stream().wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.out = step_fn()

    def __call__(self):
        self.graph.replay()
        return self.out


@torch.no_grad()
def eval_split(model, data, edge_index, mask):
    model.eval()
    logits = model(data.x, edge_index, data.timestep if _model_uses_time_embed(model) else None)
    probs = torch.softmax(logits, dim=1)[:, 1].detach().cpu().numpy()
    y = data.y.detach().cpu().numpy()
    m = mask.detach().cpu().numpy()
    return y[m], probs[m], logits


# ----------------------------------------------------------------------------- metrics (src/utils/metrics.py)
from .metrics import pr_auc_illicit  # noqa: E402  (src/utils/metrics.py restated)


def _metrics(y_bin, p, thr, cfg) -> Dict:
    """Test-split metrics of main (src/train_gnn.py:466-519) via metrics.py."""
    from . import metrics as M

    k = cfg.get("topk", 100)
    two = len(np.unique(y_bin)) > 1
    return dict(
        pr_auc_illicit=M.pr_auc_illicit(y_bin, p),
        roc_auc=M.roc_auc_illicit(y_bin, p) if two else float("nan"),
        f1_illicit_at_thr=M.f1_at_threshold(y_bin, p, thr),
        threshold=float(thr),
        precision_at_k=M.precision_at_k(y_bin, p, k) if len(p) else 0.0,
        recall_at_precision=M.recall_at_precision(y_bin, p, cfg.get("precision_target", 0.90)),
        ece=M.expected_calibration_error(y_bin, p),
        n_test=int(len(y_bin)),
    )


def _threshold(y_bin, p, cfg) -> float:
    """Decision threshold (src/train_gnn.py:466-483): precision target if set, else max F1."""
    from . import metrics as M

    target = cfg.get("precision_target", 0.0)
    if target and target > 0:
        return M.pick_threshold_for_precision(y_bin, p, target)
    return M.pick_threshold_max_f1(y_bin, p)[0]


# ----------------------------------------------------------------------------- data
def load_data(cfg: Dict) -> GraphData:
    path = cfg.get("graph_file") or os.path.join(cfg.get("processed_dir", "data/processed"), "graph.npz")
    if os.path.exists(path):
        return load_graph(path)
    syn = cfg.get("synthetic")
    if syn is None:
        raise RuntimeError(
            f"{path} not found.  Provide a PyG-free graph (dataset_elliptic.save_graph) or set "
            "`synthetic: {}` to train on the seeded Elliptic-shape generator."
        )
    return synthetic_elliptic(**(syn if isinstance(syn, dict) else {}))


def main(cfg: Dict) -> Dict:
    set_seed(cfg.get("seed", 42))
    outdir = os.path.join(cfg.get("output_root", "outputs"), "gnn", cfg["run_name"])
    os.makedirs(outdir, exist_ok=True)
    device = get_device(cfg)
    use_amp = bool(cfg.get("amp", True))
    scaler = torch.amp.GradScaler(device=device.type, enabled=use_amp)

    data = prepare_inputs(load_data(cfg), cfg)
    data = data.to(device)
    ei = data.edge_index
    model = build_model(cfg["arch"], data.x.size(1), cfg).to(device)
    opt = make_optimizer(model, cfg, device, use_amp)
    cw = class_weight(data.y[data.train_mask].cpu()) if cfg.get("class_weight_pos", "auto") == "auto" \
        else torch.tensor([1.0, float(cfg["class_weight_pos"])], dtype=torch.float32)
    t_train = data.timestep[data.train_mask]
    loss_fn = _make_loss_fn(cfg, cw, model, int(t_train.min()), int(t_train.max()))

    best_val, best_state, bad = -1.0, None, 0
    patience = cfg.get("patience", 20)
    log_path = os.path.join(outdir, "training_log.csv")
    with open(log_path, "w", newline="") as f:
        csv.writer(f).writerow(["epoch", "train_loss", "val_pr_auc"])
    for epoch in range(1, cfg["max_epochs"] + 1):
        loss = train_epoch(model, data, ei, opt, loss_fn, scaler, use_amp, cfg, device)
        y_val, p_val, _ = eval_split(model, data, ei, data.val_mask)
        pr_val = 0.0 if y_val.size == 0 else pr_auc_illicit((y_val == 1).astype(int), p_val)
        with open(log_path, "a", newline="") as f:
            csv.writer(f).writerow([epoch, f"{loss:.6f}", f"{pr_val:.6f}"])
        if pr_val > best_val:
            best_val, bad = pr_val, 0
            best_state = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
        else:
            bad += 1
        if epoch % 10 == 0 or epoch == 1:
            print(f"Epoch {epoch:4d} | loss {loss:.4f} | val PR-AUC(illicit) {pr_val:.4f} (best {best_val:.4f})")
        if bad >= patience:
            print("Early stopping.")
            break
    if best_state is not None:
        model.load_state_dict({k: v.to(device) for k, v in best_state.items()})

    T = None
    if bool(cfg.get("calibrate_temperature", True)):
        _, _, lv = eval_split(model, data, ei, data.val_mask)
        Tp = torch.ones(1, device=device, requires_grad=True)
        lbfgs = torch.optim.LBFGS([Tp], lr=0.1, max_iter=1000)
        lv, yv = lv[data.val_mask].detach(), data.y[data.val_mask]

        def closure():
            lbfgs.zero_grad()
            l = F.cross_entropy(lv / Tp, yv.long())
            l.backward()
            return l

        lbfgs.step(closure)
        T = Tp.detach()

    def get_probs(edge_index_eval):
        model.eval()
        with torch.no_grad():
            lg = model(data.x, edge_index_eval, data.timestep if _model_uses_time_embed(model) else None)
            if T is not None:
                lg = lg / T
            return torch.softmax(lg, dim=1)[:, 1].cpu().numpy()

    probs = get_probs(ei)
    y_np = data.y.cpu().numpy()
    vm, tm = data.val_mask.cpu().numpy(), data.test_mask.cpu().numpy()
    ts = data.timestep.cpu().numpy()
    for split, m in (("val", vm), ("test", tm)):
        np.save(os.path.join(outdir, f"scores_{split}.npy"), probs[m])
        np.save(os.path.join(outdir, f"y_{split}.npy"), y_np[m])
        np.save(os.path.join(outdir, f"node_idx_{split}.npy"), np.where(m)[0])
        np.save(os.path.join(outdir, f"timestep_{split}.npy"), ts[m])
    y_val, p_val = (y_np[vm] == 1).astype(int), probs[vm]
    y_te, p_te = (y_np[tm] == 1).astype(int), probs[tm]
    thr = _threshold(y_val, p_val, cfg) if cfg.get("use_val_for_thresholds", True) else _threshold(y_te, p_te, cfg)
    metrics = _metrics(y_te, p_te, thr, cfg) if y_te.size else {}
    metrics["best_val_pr_auc"] = best_val
    torch.save(model.state_dict(), os.path.join(outdir, "best.ckpt"))
    with open(os.path.join(outdir, "metrics.json"), "w") as f:
        json.dump(metrics, f, indent=2)
    with open(os.path.join(outdir, "config_used.yaml"), "w") as f:
        yaml.safe_dump(cfg, f)
    print(json.dumps(metrics, indent=2))
    return metrics


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=str, required=True)
    args = ap.parse_args()
    with open(args.config) as f:
        main(yaml.safe_load(f))
