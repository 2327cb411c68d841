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
The mini-batch path (:212-245, :260-276, :329-348) runs on loader.NeighborLoader (K11 sampling).
"""
from __future__ import annotations

import argparse
import contextlib
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
from .distributed import GradBucket, convert_sync_batchnorm, gather_rows, shard_graph
from . import fused
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


def _make_loss_fn(cfg: Dict, cw: torch.Tensor, model, t_min: int, t_max: int, world: int = 1):
    """src/train_gnn.py:136-183.  ``world`` > 1 (timestep-partitioned ranks): the embedding L2
    term is added once per rank, so each rank adds 1/world of it (the all-reduced gradient and
    loss then carry it once)."""
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
            loss = loss + (embed_l2 / world) * model.time_emb.weight.pow(2).mean()
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

    def target(y_all, mask, denom):
        """Context for the training forward whose loss is ``full(logits, y_all, mask, denom)``:
        the forward may compute that masked CE itself (train_ops.fused_ce_target — the fused SAGE
        output layer does, in its aggregation's launch); a no-op for the other loss variants."""
        if not (loss_fn.plain and y_all.is_cuda and denom is not None):
            return contextlib.nullcontext()
        from .train_ops import fused_ce_target

        w = cw_dev.get(y_all.device)
        if w is None:
            w = cw_dev[y_all.device] = cw.to(y_all.device)
        return fused_ce_target(y_all, mask, w, denom)

    loss_fn.plain = not focal and scheme == "none" and embed_l2 == 0.0
    loss_fn.full = full
    loss_fn.target = target
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


def amp_is_exact(model) -> bool:
    """True when the model's whole training forward runs as one fp32 libgnnmp autograd node (fused
    SAGENet / GCNNet): autocast changes nothing inside it (custom_fwd casts to fp32), and
    GradScaler's power-of-two scale and unscale are exact on its fp32 gradients, so the reference's
    AMP step (src/train_gnn.py:192-207) equals the unscaled step except for GradScaler's skip of a
    non-finite update — which ClipAdam(skip_nonfinite) reproduces."""
    from . import fused
    from .gnn import GCNNet, SAGENet

    if isinstance(model, SAGENet):
        return model.fused and fused.fusable(model)
    if isinstance(model, GCNNet):
        return model.fused and fused.gcn_fusable(model)
    return False


def make_optimizer(model, cfg: Dict, device, use_amp: bool):
    """Adam(lr, weight_decay) (src/train_gnn.py:357).  On the GPU: ClipAdam, the fused
    clip_grad_norm_(grad_clip) + Adam step (train_ops.py), when one launch pair covers the
    parameters (≤ ADAM_MAX_TENSORS tensors) and, under AMP, when the AMP step is exact on the
    model (amp_is_exact: ClipAdam then also takes GradScaler's skip of a non-finite update);
    otherwise torch.optim.Adam (train_epoch then clips with clip_grad_norm_ as the reference does)."""
    if device.type == "cuda" and (not use_amp or amp_is_exact(model)):
        from .train_ops import ClipAdam
        if ClipAdam.supports(model.parameters()):
            clip = cfg.get("grad_clip", 0)
            return ClipAdam(model.parameters(), lr=cfg["lr"], weight_decay=cfg["weight_decay"],
                            max_norm=float(clip) if clip and clip > 0 else None, skip_nonfinite=use_amp)
    return torch.optim.Adam(model.parameters(), lr=cfg["lr"], weight_decay=cfg["weight_decay"])


def train_epoch(model, data, edge_index, optimizer, loss_fn, scaler, use_amp, cfg, device, sync=True,
                denom=None, bucket=None, dist=None):
    """One full-batch step (src/train_gnn.py:187-209).  ``sync=False`` keeps the loss on device.

    Timestep-partitioned data parallelism: ``denom`` is the GLOBAL train count (the per-rank
    loss is sum/denom, so the ranks' losses and gradients add up to the single-device .mean(),
    :175) and ``bucket`` (distributed.GradBucket) all-reduces every gradient in one collective
    before the clip and the optimizer step, so every rank applies the same update."""
    model.train()
    optimizer.zero_grad(set_to_none=bucket is None)
    if denom is None:
        denom = getattr(data, "n_train", None)
    # AMP on an fp32 libgnnmp model (amp_is_exact): the fused step, GradScaler's scale / unscale
    # left out (exact on fp32 gradients) and its skip of a non-finite update done by ClipAdam
    amp_fused = use_amp and getattr(optimizer, "skip_nonfinite", False)
    fused_ce = getattr(loss_fn, "plain", False) and (not use_amp or amp_fused) and denom is not None
    with _autocast(device, use_amp):
        with (loss_fn.target(data.y, data.train_mask, denom) if fused_ce else contextlib.nullcontext()):
            logits = model(data.x, edge_index, data.timestep if _model_uses_time_embed(model) else None)
        t_idx = _rows(data.timestep, data, "train") if cfg.get("time_loss_weighting", "none") != "none" else None
        if (getattr(loss_fn, "plain", False) and logits.is_cuda and logits.dtype == torch.float32
                and (not use_amp or amp_fused)):
            loss = loss_fn.full(logits, data.y, data.train_mask, denom=denom)
        else:
            loss = loss_fn(_rows(logits, data, "train"), _rows(data.y, data, "train"), t_idx,
                           denom=denom if bucket is not None else None)
    if (scaler.is_enabled() and not amp_fused) or not loss.is_cuda:
        scaler.scale(loss).backward()
    else:  # = loss.backward(): a persistent unit gradient (no fill kernel; the fused CE skips `* g`)
        from .train_ops import unit_gradient

        loss.backward(unit_gradient(loss.device))
    if bucket is not None:
        bucket.allreduce_(dist)
    if cfg.get("grad_clip", 0) and cfg["grad_clip"] > 0 and not _clips_itself(optimizer):
        scaler.unscale_(optimizer)
        torch.nn.utils.clip_grad_norm_(model.parameters(), cfg["grad_clip"])
    if amp_fused:
        optimizer.step()
    else:
        scaler.step(optimizer)
        scaler.update()
    optimizer.zero_grad(set_to_none=bucket is None)
    if bucket is not None:
        loss = loss.detach().clone()
        dist.all_reduce(loss)  # the global loss (sum of the ranks' partial means)
    return float(loss.item()) if sync else loss.detach()


def train_epoch_minibatch(model, loader, optimizer, loss_fn, scaler, use_amp, cfg, device):
    """One epoch over NeighborLoader batches (src/train_gnn.py:212-245): the loss is taken on the
    first ``batch.batch_size`` rows (the seeds), one optimizer step per batch; returns the
    seed-weighted mean loss."""
    model.train()
    total_loss, total_examples = 0.0, 0
    uses_t = _model_uses_time_embed(model)
    weighted = cfg.get("time_loss_weighting", "none") != "none"
    for batch in loader:
        batch = batch.to(device)
        bs = int(batch.batch_size)
        optimizer.zero_grad(set_to_none=True)
        with _autocast(device, use_amp):
            logits = model(batch.x, batch.edge_index, batch.timestep if uses_t else None)
            t_idx = batch.timestep[:bs] if weighted else None
            loss = loss_fn(logits[:bs], batch.y[:bs], t_idx)
        scaler.scale(loss).backward()
        if cfg.get("grad_clip", 0) and cfg["grad_clip"] > 0 and not _clips_itself(optimizer):
            scaler.unscale_(optimizer)
            torch.nn.utils.clip_grad_norm_(model.parameters(), cfg["grad_clip"])
        scaler.step(optimizer)
        scaler.update()
        optimizer.zero_grad(set_to_none=True)
        total_loss += float(loss.item()) * bs
        total_examples += bs
    return 0.0 if total_examples == 0 else float(total_loss / total_examples)


@torch.no_grad()
def eval_val_minibatch(model, loader, device):
    """src/train_gnn.py:260-276: P(illicit) of every batch's seed rows, concatenated."""
    model.eval()
    ys, ps = [], []
    uses_t = _model_uses_time_embed(model)
    for batch in loader:
        batch = batch.to(device)
        bs = int(batch.batch_size)
        logits = model(batch.x, batch.edge_index, batch.timestep if uses_t else None)[:bs]
        ps.append(torch.softmax(logits, dim=1)[:, 1].detach().cpu())
        ys.append(batch.y[:bs].detach().cpu())
    if not ys:
        return np.array([]), np.array([])
    return torch.cat(ys).numpy(), torch.cat(ps).numpy()


class CapturedStep:
    """A training step captured into HIP graphs and replayed (torch.cuda.CUDAGraph).

    ``step_fn`` must be capture-safe: static input tensors, no host syncs, an optimizer whose
    state advances on the device (ClipAdam, or torch Adam with ``capturable=True``).  The fused
    SAGE / GAT paths switch their dropout seed to a device counter under capture, so every replay
    draws a new mask.  Replaying removes the host's per-kernel launch cost and the gaps between
    kernels.

    Collectives: RCCL all-reduces (backend "nccl": SyncBN statistics, the gradient bucket) are
    stream-captured like any kernel, so an N>1 step over RCCL is ONE graph (``step_fn`` calls
    them; the communicator is set up by the eager warm-up before capture).  Split form (``mid``
    and ``tail`` given), for CPU-side collectives (gloo): ``step_fn`` (forward + backward) is
    graph A, ``mid`` runs eagerly (the gradient all-reduce) and ``tail`` (the optimizer step) is
    graph B.

    ``defer_loss`` (off by default): the fused CE's loss scalar is finished at the step's end —
    inside ClipAdam's launch, or by a launch recorded at the end of the capture — one launch fewer
    per replay.  Only for a ``step_fn`` that reads the loss after the optimizer step (returns it,
    as bench.py and train_epoch do): read before it, the loss tensor still holds the previous
    replay's value.  The CE partials such a loss reads at the step's end are held here
    (``self._held``) for the graph's lifetime.
    """

    def __init__(self, step_fn, warmup: int = 3, mid=None, tail=None, defer_loss: bool = False):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                step_fn()
                if mid is not None:
                    mid()
                if tail is not None:
                    tail()
        torch.cuda.current_stream().wait_stream(side)
        self.mid = mid
        self.graph = torch.cuda.CUDAGraph()
        self.tail_graph = None
        # the dropout counter's per-step bump runs at the step's end (fused.deferred_seed_bumps):
        # inside ClipAdam's launch when the step has one, else as an add recorded here
        with fused.deferred_seed_bumps(defer_loss=defer_loss) as dctx:
            # thread-local capture mode: the process group's watchdog thread keeps querying the events
            # of earlier (eager) collectives while this thread captures; in the default global mode
            # such a query from another thread invalidates the capture (hipErrorStreamCaptureUnsupported)
            with torch.cuda.graph(self.graph, capture_error_mode="thread_local"):
                self.out = step_fn()
                if tail is None:
                    fused.flush_seed_bumps()
            if tail is not None:
                self.tail_graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self.tail_graph, pool=self.graph.pool(), capture_error_mode="thread_local"):
                    tail()
                    fused.flush_seed_bumps()
        self._held = list(dctx.held)  # buffers a replay still reads at its end (deferred loss partials)

    def __call__(self):
        self.graph.replay()
        if self.mid is not None:
            self.mid()
        if self.tail_graph is not None:
            self.tail_graph.replay()
        return self.out


@torch.no_grad()
def eval_split(model, data, edge_index, mask, dist=None, num_nodes=None):
    """src/train_gnn.py:248-257.  Partitioned (``dist`` given, ``data`` a shard): every rank runs
    its own timesteps and the probabilities / labels are gathered over the global node order
    (``num_nodes`` rows); ``mask`` is then the GLOBAL mask (host or device)."""
    model.eval()
    logits = model(data.x, edge_index, data.timestep if _model_uses_time_embed(model) else None)
    if dist is not None:
        logits = gather_rows(logits.float(), data.nodes, num_nodes, dist)
        y = gather_rows(data.y, data.nodes, num_nodes, dist)
    else:
        y = data.y
    probs = torch.softmax(logits, dim=1)[:, 1].detach().cpu().numpy()
    y = y.detach().cpu().numpy()
    m = mask.detach().cpu().numpy()
    return y[m], probs[m], logits


class RunLogger:
    """``training_log.csv`` (epoch, train_loss, val_pr_auc) as src/utils/logger.py:5-27 writes it,
    plus the TensorBoard scalars when tensorboard is importable (it is optional here)."""

    def __init__(self, outdir: str):
        os.makedirs(outdir, exist_ok=True)
        self.csv_path = os.path.join(outdir, "training_log.csv")
        if not os.path.exists(self.csv_path):
            with open(self.csv_path, "w", newline="") as f:
                csv.writer(f).writerow(["epoch", "train_loss", "val_pr_auc"])
        self.tb = None
        try:
            from torch.utils.tensorboard import SummaryWriter
            self.tb = SummaryWriter(log_dir=os.path.join(outdir, "tb"))
        except Exception:  # tensorboard absent: CSV only
            self.tb = None

    def log_epoch(self, epoch: int, train_loss: float, val_pr_auc: float) -> None:
        with open(self.csv_path, "a", newline="") as f:
            csv.writer(f).writerow([epoch, f"{train_loss:.6f}", f"{val_pr_auc:.6f}"])
        if self.tb is not None:
            self.tb.add_scalar("loss/train", train_loss, epoch)
            self.tb.add_scalar("val/pr_auc_illicit", val_pr_auc, epoch)

    def close(self) -> None:
        if self.tb is not None:
            self.tb.flush()
            self.tb.close()


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


def _max_f1_threshold(y_bin, p) -> float:
    """use_val_for_thresholds false: max-F1 threshold on the test split (src/train_gnn.py:473-474)."""
    from . import metrics as M

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


def _init_distributed(cfg: Dict):
    """One process per GPU under torch.distributed.run (WORLD_SIZE/RANK/LOCAL_RANK from the env).

    New optional keys: ``world_size`` (must equal WORLD_SIZE when given),
    ``partition`` ('timestep': whole timesteps per rank — exact, the graph is block-diagonal in
    time, src/data/dataset_elliptic.py:235-243) and ``dist_backend`` ('nccl' = RCCL, default;
    'gloo' for tests).  Returns (dist or None, world, rank)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    want = int(cfg.get("world_size", world) or 1)
    if want != world:
        raise RuntimeError(f"world_size={want} but WORLD_SIZE={world}: launch with "
                           f"python -m torch.distributed.run --nproc-per-node {want} ...")
    if world == 1:
        return None, 1, 0
    if cfg.get("partition", "timestep") != "timestep":
        raise ValueError(f"partition={cfg.get('partition')!r}: only 'timestep' partitioning is exact")
    import torch.distributed as dist

    rank = int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        torch.cuda.set_device(local % torch.cuda.device_count())
    if not dist.is_initialized():
        backend = cfg.get("dist_backend", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", torch.cuda.current_device()))
        else:
            dist.init_process_group(backend)
    return dist, world, rank


def per_timestep_pr_auc(y_te: np.ndarray, p_te: np.ndarray, test_ts: np.ndarray) -> Dict:
    """``test_pr_auc_by_time`` and ``pr_auc_last{1,3,5}`` of metrics.json (src/train_gnn.py:497-519):
    PR-AUC of each test timestep in chronological order, and the means of the last 1/3/5."""
    out: Dict = {}
    if test_ts.size == 0:
        return out
    pr_by_t = []
    for t in sorted(set(int(v) for v in test_ts.tolist())):
        idx = test_ts == t
        pr_by_t.append(float("nan") if idx.sum() == 0 else pr_auc_illicit((y_te[idx] == 1).astype(int), p_te[idx]))
    out["test_pr_auc_by_time"] = pr_by_t
    if pr_by_t:
        out["pr_auc_last1"] = float(pr_by_t[-1])
        if len(pr_by_t) >= 3:
            out["pr_auc_last3"] = float(sum(pr_by_t[-3:]) / 3)
        if len(pr_by_t) >= 5:
            out["pr_auc_last5"] = float(sum(pr_by_t[-5:]) / 5)
    return out


def hub_edge_mask(edge_index: torch.Tensor, num_nodes: int, frac: float):
    """Edges kept by the hub ablation of main (src/train_gnn.py:526-539): the int(frac·N) nodes of
    highest in+out degree (torch.topk, as the reference) lose every incident edge.
    Returns (hub flags [N] bool, kept-edge mask [E] bool, number of hubs); host tensors."""
    ei = edge_index.detach().cpu()
    num_hubs = int(frac * float(num_nodes))
    deg = torch.bincount(ei[0], minlength=num_nodes) + torch.bincount(ei[1], minlength=num_nodes)
    hubs = torch.zeros(num_nodes, dtype=torch.bool)
    if num_hubs > 0:
        hubs[torch.topk(deg, num_hubs).indices] = True
    return hubs, ~(hubs[ei[0]] | hubs[ei[1]]), num_hubs


def main(cfg: Dict) -> Dict:
    """src/train_gnn.py:282-564 on libgnnmp, single GPU or timestep-partitioned over ranks."""
    dist, world, rank = _init_distributed(cfg)
    set_seed(cfg.get("seed", 42))  # same seed on every rank: identical initial weights
    is_main = rank == 0
    outdir = os.path.join(cfg.get("output_root", "outputs"), "gnn", cfg["run_name"])
    logger = RunLogger(outdir) if is_main else None
    device = get_device(cfg)
    use_mini_batch = bool(cfg.get("mini_batch", False))
    if use_mini_batch and dist is not None:
        raise NotImplementedError("mini_batch with world_size > 1: the reference's NeighborLoader path is "
                                  "single-device (src/train_gnn.py:329-348)")
    use_amp = device.type == "cuda" and bool(cfg.get("amp", True))  # src/train_gnn.py:291
    scaler = torch.amp.GradScaler(device=device.type, enabled=use_amp)

    full = prepare_inputs(load_data(cfg), cfg)  # host: masks window, time scalar, symmetrize
    N = full.num_nodes
    n_train = int(full.n_train)
    local = shard_graph(full, world, rank) if dist is not None else full
    data = local.to(device)
    if device.type == "cuda":
        from .planes import register_input

        register_input(data.x)  # constant node features: layer-1 GEMMs on its split image
    ei = data.edge_index
    model = build_model(cfg["arch"], data.x.size(1), cfg).to(device)
    bucket = None
    if dist is not None:
        convert_sync_batchnorm(model, dist)  # BatchNorm over all N nodes (gnn.py:188-189)
        bucket = GradBucket(model)
    opt = make_optimizer(model, cfg, device, use_amp)
    cw = class_weight(full.y[full.train_mask]) if cfg.get("class_weight_pos", "auto") == "auto" \
        else torch.tensor([1.0, float(cfg["class_weight_pos"])], dtype=torch.float32)
    t_train = full.timestep[full.train_mask]
    loss_fn = _make_loss_fn(cfg, cw, model, int(t_train.min()), int(t_train.max()), world)
    gmask = (lambda name: getattr(full, name)) if dist is not None else (lambda name: getattr(data, name))
    ev = dict(dist=dist, num_nodes=N) if dist is not None else {}

    train_loader = val_loader = None
    if use_mini_batch:  # src/train_gnn.py:329-348 (loaders over the symmetrized graph)
        from .loader import NeighborLoader
        fanout = cfg.get("fanout", [10, 10])
        bsz = int(cfg.get("batch_size", 8192))
        train_loader = NeighborLoader(data, num_neighbors=fanout, batch_size=bsz,
                                      input_nodes=data.train_mask.nonzero().view(-1), shuffle=True)
        val_loader = NeighborLoader(data, num_neighbors=fanout, batch_size=bsz,
                                    input_nodes=data.val_mask.nonzero().view(-1), shuffle=False)

    best_val, best_state, bad = -1.0, None, 0
    patience = cfg.get("patience", 20)
    for epoch in range(1, cfg["max_epochs"] + 1):
        if use_mini_batch:
            loss = train_epoch_minibatch(model, train_loader, opt, loss_fn, scaler, use_amp, cfg, device)
            y_val, p_val = eval_val_minibatch(model, val_loader, device)
        else:
            loss = train_epoch(model, data, ei, opt, loss_fn, scaler, use_amp, cfg, device, denom=n_train,
                               bucket=bucket, dist=dist)
            y_val, p_val, _ = eval_split(model, data, ei, gmask("val_mask"), **ev)
        pr_val = 0.0 if y_val.size == 0 else pr_auc_illicit((y_val == 1).astype(int), p_val)
        if logger is not None:
            logger.log_epoch(epoch, loss, pr_val)
        if pr_val > best_val:
            best_val, bad = pr_val, 0
            best_state = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
        else:
            bad += 1
        if is_main and (epoch % 10 == 0 or epoch == 1):
            print(f"Epoch {epoch:4d} | loss {loss:.4f} | val PR-AUC(illicit) {pr_val:.4f} (best {best_val:.4f})")
        if bad >= patience:
            if is_main:
                print("Early stopping.")
            break
    if best_state is not None:
        model.load_state_dict({k: v.to(device) for k, v in best_state.items()})

    T = None
    if bool(cfg.get("calibrate_temperature", True)):  # TemperatureScaler.fit (src/utils/calibrate.py:8-30)
        _, _, lv = eval_split(model, data, ei, gmask("val_mask"), **ev)
        vm_dev = gmask("val_mask").to(lv.device)
        yv = (gather_rows(data.y, data.nodes, N, dist) if dist is not None else data.y)[vm_dev]
        Tp = torch.ones(1, device=device, requires_grad=True)
        lbfgs = torch.optim.LBFGS([Tp], lr=0.1, max_iter=1000)
        lv = lv[vm_dev].detach()

        def closure():
            lbfgs.zero_grad()
            l = F.cross_entropy(lv / Tp, yv.long())
            l.backward()
            return l

        lbfgs.step(closure)
        T = Tp.detach()
        if dist is not None:
            dist.broadcast(T, 0)  # one temperature for every rank

    def get_probs(edge_index_eval):
        model.eval()
        with torch.no_grad():
            lg = model(data.x, edge_index_eval, data.timestep if _model_uses_time_embed(model) else None)
            if dist is not None:
                lg = gather_rows(lg.float(), data.nodes, N, dist)
            if T is not None:
                lg = lg / T
            return torch.softmax(lg, dim=1)[:, 1].cpu().numpy()

    probs = get_probs(ei)
    y_np = full.y.numpy() if dist is not None else data.y.cpu().numpy()
    vm, tm = gmask("val_mask").cpu().numpy(), gmask("test_mask").cpu().numpy()
    ts = full.timestep.numpy() if dist is not None else data.timestep.cpu().numpy()
    y_val, p_val = (y_np[vm] == 1).astype(int), probs[vm]
    y_te, p_te = (y_np[tm] == 1).astype(int), probs[tm]
    thr = _threshold(y_val, p_val, cfg) if cfg.get("use_val_for_thresholds", True) \
        else _max_f1_threshold(y_te, p_te)
    metrics = _metrics(y_te, p_te, thr, cfg) if y_te.size else {}
    metrics["best_val_pr_auc"] = best_val
    metrics.update(per_timestep_pr_auc(y_np[tm], p_te, ts[tm]))

    frac = float(cfg.get("ablate_hubs_frac", 0.0))
    metrics_hub = None
    if frac > 0:  # src/train_gnn.py:525-558: forward again without the hubs' edges
        hubs, keep, num_hubs = hub_edge_mask(full.edge_index, N, frac)
        if dist is not None:  # this rank's edges, through its nodes' global ids
            nodes = local.nodes
            lei = local.edge_index
            keep_l = ~(hubs[nodes[lei[0]]] | hubs[nodes[lei[1]]])
            ei_abl = lei[:, keep_l].to(device)
        else:
            ei_abl = full.edge_index[:, keep].to(device)
        p_abl = get_probs(ei_abl)[tm]
        metrics_hub = _metrics(y_te, p_abl, thr, cfg) if y_te.size else {}
        metrics_hub.update(n_hubs=int(num_hubs), hub_fraction=frac, n_edges_remaining=int(keep.sum()))

    if is_main:
        for split, m in (("val", vm), ("test", tm)):
            np.save(os.path.join(outdir, f"scores_{split}.npy"), probs[m])
            np.save(os.path.join(outdir, f"y_{split}.npy"), y_np[m])
            np.save(os.path.join(outdir, f"node_idx_{split}.npy"), np.where(m)[0])
            np.save(os.path.join(outdir, f"timestep_{split}.npy"), ts[m])
        torch.save(model.state_dict(), os.path.join(outdir, "best.ckpt"))
        with open(os.path.join(outdir, "metrics.json"), "w") as f:
            json.dump(metrics, f, indent=2)
        if metrics_hub is not None:
            with open(os.path.join(outdir, "metrics_hub_removed.json"), "w") as f:
                json.dump(metrics_hub, f, indent=2)
        with open(os.path.join(outdir, "config_used.yaml"), "w") as f:
            yaml.safe_dump(cfg, f)
        logger.close()
        print(json.dumps(metrics, indent=2))
    return metrics


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=str, required=True)
    args = ap.parse_args()
    with open(args.config) as f:
        main(yaml.safe_load(f))
