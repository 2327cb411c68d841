"""Graph container, temporal masks and the synthetic Elliptic-shape generator.

The reference's loader (src/data/dataset_elliptic.py:49-265) turns the Elliptic CSVs into
a PyG ``Data(x[N,165] f32, edge_index[2,E] i64, y[N] i64, timestep[N] i64)`` and drops
every edge whose endpoints lie in different timesteps (:235-243).  The CSVs are git-LFS
pointers in the reference (data/raw/*.csv, .gitattributes:1), so this build runs on a
seeded synthetic graph of the same shape:

  N = 203,769 nodes in 49 contiguous timestep blocks; E0 = 234,355 directed
  intra-timestep edges (no self loops); x ~ N(0,1) [N,165] f32; labels 4,545 illicit,
  42,019 licit, the rest unknown (-1).  In-degree: 'uniform' or 'powerlaw' (Chung-Lu
  weights w = 1/u, P(deg > k) ~ 1/k: hubs of a few hundred edges, as in Elliptic).

``GraphData`` replaces PyG's ``Data`` (attribute access, ``.to(device)``), so the
training loop needs no torch_geometric.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, Optional

import numpy as np
import torch

ELLIPTIC_NODES = 203_769
ELLIPTIC_EDGES = 234_355
ELLIPTIC_TIMESTEPS = 49
ELLIPTIC_FEATS = 165
ELLIPTIC_ILLICIT = 4_545
ELLIPTIC_LICIT = 42_019


class GraphData:
    """Minimal stand-in for torch_geometric.data.Data: named tensors + ``to``."""

    def __init__(self, **tensors):
        for k, v in tensors.items():
            setattr(self, k, v)

    def keys(self):
        return [k for k, v in vars(self).items() if isinstance(v, torch.Tensor)]

    @property
    def num_nodes(self) -> int:
        return int(self.x.size(0))

    def to(self, device) -> "GraphData":
        return GraphData(**{k: (v.to(device) if isinstance(v, torch.Tensor) else v) for k, v in vars(self).items()})

    def __repr__(self) -> str:
        parts = [f"{k}={list(v.shape)}" for k, v in vars(self).items() if isinstance(v, torch.Tensor)]
        return f"GraphData({', '.join(parts)})"


def make_temporal_masks(data: GraphData, t_train_end: int, t_val_end: int,
                        train_window_k: Optional[int] = None) -> GraphData:
    """Train/val/test masks over labelled nodes (reference: src/data/dataset_elliptic.py:268-290).

    train: t <= t_train_end (or the last ``train_window_k`` train timesteps); val: (t_train_end,
    t_val_end]; test: > t_val_end.  Unlabelled (y < 0) nodes are in no mask.
    """
    y, t = data.y, data.timestep
    labelled = y >= 0
    lo = 1 if train_window_k is None else max(1, t_train_end - int(train_window_k) + 1)
    data.train_mask = (t >= lo) & (t <= t_train_end) & labelled
    data.val_mask = (t > t_train_end) & (t <= t_val_end) & labelled
    data.test_mask = (t > t_val_end) & labelled
    return data


def _split_counts(total: int, weights: np.ndarray) -> np.ndarray:
    w = weights / weights.sum()
    c = np.floor(total * w).astype(np.int64)
    rem = total - int(c.sum())
    c[np.argsort(-(total * w - c), kind="stable")[:rem]] += 1
    return c


def synthetic_elliptic(num_nodes: int = ELLIPTIC_NODES, num_edges: int = ELLIPTIC_EDGES,
                       num_timesteps: int = ELLIPTIC_TIMESTEPS, num_feats: int = ELLIPTIC_FEATS,
                       degree: str = "powerlaw", seed: int = 42, num_illicit: Optional[int] = None,
                       num_licit: Optional[int] = None, feature_dtype=np.float32) -> GraphData:
    """Seeded Elliptic-shaped graph (block-diagonal over timesteps, no cross-timestep edges)."""
    if degree not in ("uniform", "powerlaw"):
        raise ValueError(f"degree must be 'uniform' or 'powerlaw', got {degree!r}")
    rng = np.random.default_rng(seed)
    T = int(num_timesteps)
    sizes = _split_counts(num_nodes, rng.uniform(0.5, 1.5, size=T))
    offs = np.concatenate([[0], np.cumsum(sizes)])
    ecounts = _split_counts(num_edges, sizes.astype(np.float64))
    timestep = np.repeat(np.arange(1, T + 1, dtype=np.int64), sizes)
    srcs, dsts = [], []
    for t in range(T):
        n, e, o = int(sizes[t]), int(ecounts[t]), int(offs[t])
        if e == 0 or n == 0:
            continue
        s = rng.integers(0, n, size=e)
        if degree == "uniform":
            d = rng.integers(0, n, size=e)
        else:
            w = 1.0 / rng.uniform(1e-3, 1.0, size=n)  # Chung-Lu weights, heavy tail capped at 1000x
            d = rng.choice(n, size=e, p=w / w.sum())
        if n > 1:  # Elliptic has no self loops: shift a colliding target to the next node
            hit = s == d
            d[hit] = (d[hit] + 1) % n
        srcs.append(s + o)
        dsts.append(d + o)
    src = np.concatenate(srcs) if srcs else np.zeros(0, np.int64)
    dst = np.concatenate(dsts) if dsts else np.zeros(0, np.int64)
    perm = rng.permutation(src.size)  # edge-list order is arbitrary in the CSV
    edge_index = np.stack([src[perm], dst[perm]]).astype(np.int64)
    x = rng.standard_normal(size=(num_nodes, num_feats), dtype=np.float32).astype(feature_dtype, copy=False)
    n_ill = ELLIPTIC_ILLICIT if num_illicit is None else num_illicit
    n_lic = ELLIPTIC_LICIT if num_licit is None else num_licit
    if num_illicit is None and num_nodes != ELLIPTIC_NODES:  # keep Elliptic's label fractions
        n_ill = int(round(num_nodes * ELLIPTIC_ILLICIT / ELLIPTIC_NODES))
        n_lic = int(round(num_nodes * ELLIPTIC_LICIT / ELLIPTIC_NODES))
    y = np.full(num_nodes, -1, dtype=np.int64)
    lab = rng.permutation(num_nodes)[: n_ill + n_lic]
    y[lab[:n_ill]] = 1
    y[lab[n_ill:]] = 0
    return GraphData(
        x=torch.from_numpy(x),
        edge_index=torch.from_numpy(edge_index),
        y=torch.from_numpy(y),
        timestep=torch.from_numpy(timestep),
    )


def prepare_inputs(data: GraphData, cfg: Dict, split: Optional[Dict] = None) -> GraphData:
    """The reference's data prep before the epoch loop (src/train_gnn.py:300-326).

    Rolling train window (make_temporal_masks with t_train_end / t_val_end inferred from the
    existing masks, or from ``split``), ``use_time_scalar`` (x <- [x, t/max t] when no time
    embedding), ``symmetrize_edges`` (concatenate the flipped edges; no dedup).
    """
    split = split or {"t_train_end": 34, "t_val_end": 43}
    if not hasattr(data, "train_mask"):
        make_temporal_masks(data, split["t_train_end"], split["t_val_end"])
    k = cfg.get("train_window_k")
    if k is not None:
        ts = data.timestep[data.train_mask]
        vs = data.timestep[data.val_mask]
        if ts.numel() == 0:
            raise RuntimeError("Train mask is empty; cannot apply rolling window.")
        if vs.numel() == 0:
            raise RuntimeError("Validation mask is empty; cannot infer t_val_end.")
        make_temporal_masks(data, int(ts.max()), int(vs.max()), int(k))
    if cfg.get("use_time_scalar", False) and cfg.get("time_embed_dim", 0) == 0:
        tnorm = (data.timestep.float() / float(data.timestep.max())).unsqueeze(1)
        data.x = torch.cat([data.x, tnorm], dim=1)
    if cfg.get("symmetrize_edges", False):
        data.edge_index = torch.cat([data.edge_index, data.edge_index.flip(0)], dim=1)
    index_masks(data)
    return data


def index_masks(data: GraphData) -> GraphData:
    """Row indices of the split masks, computed once.  ``logits[mask]`` on a device needs a
    nonzero() and a host sync every call; ``logits.index_select(0, idx)`` is the same rows in
    the same order with neither (and its backward is a scatter, not a sort)."""
    for name in ("train", "val", "test"):
        m = getattr(data, f"{name}_mask", None)
        if m is not None:
            idx = torch.nonzero(m, as_tuple=False).flatten()
            setattr(data, f"{name}_idx", idx)
            setattr(data, f"n_{name}", int(idx.numel()))  # host ints: the loss divisor needs no sync
    return data


def concat_graphs(blocks) -> GraphData:
    """Disjoint union of prepared graphs (node rows stacked, edges offset, order kept), with
    ``part_key`` = timestep + T_max·block so that whole (block, timestep) units can be
    partitioned (bench.py's weak-scaling graph: one Elliptic-shaped block per rank)."""
    keys = [k for k in blocks[0].keys() if not k.endswith("_idx")]
    out, off, tmax = {}, 0, max(int(b.timestep.max()) for b in blocks)
    eis, pk = [], []
    for bi, b in enumerate(blocks):
        eis.append(b.edge_index + off)
        pk.append(b.timestep + tmax * bi)
        off += b.num_nodes
    for k in keys:
        if k != "edge_index":
            out[k] = torch.cat([getattr(b, k) for b in blocks], dim=0)
    out["edge_index"] = torch.cat(eis, dim=1)
    out["part_key"] = torch.cat(pk)
    return index_masks(GraphData(**out))


def save_graph(path: str, data: GraphData) -> None:
    """PyG-free on-disk graph (npz of plain arrays; loadable with allow_pickle=False)."""
    np.savez(path, **{k: getattr(data, k).numpy() for k in data.keys()})


def load_graph(path: str) -> GraphData:
    with np.load(path, allow_pickle=False) as z:
        return GraphData(**{k: torch.from_numpy(z[k]) for k in z.files})


# ----------------------------------------------------------------------------- CSV ingest
_LABELS = {"class1": 1, "1": 1, "illicit": 1, "class2": 0, "2": 0, "licit": 0, "unknown": -1, "-1": -1}


def _label(v) -> int:
    """Elliptic class string/number -> 1 illicit, 0 licit, -1 unknown (dataset_elliptic.py:12-29)."""
    return _LABELS.get(str(v).strip().lower(), -1)


def _is_timestep_column(col) -> bool:
    """Integers in [1, 49] (>95 % integral): the Elliptic time index (dataset_elliptic.py:32-46)."""
    import pandas as pd

    v = pd.to_numeric(col, errors="coerce").dropna().astype(float)
    return (not v.empty) and v.min() >= 1 and v.max() <= 49 and bool((v.round() == v).mean() > 0.95)


def load_elliptic_csv(data_dir: str, features_csv: str = "elliptic_txs_features.csv",
                      classes_csv: str = "elliptic_txs_classes.csv",
                      edgelist_csv: str = "elliptic_txs_edgelist.csv") -> GraphData:
    """Elliptic CSVs -> GraphData(x, edge_index, y, timestep): the reference's
    load_elliptic_as_graph (src/data/dataset_elliptic.py:49-265), without PyG.

    Nodes in features-CSV row order (a left join keeps it, :163); features = every column after
    txId, minus column 1 when it looks like the timestep (:113-140); timestep from classes.csv
    ('time_step' / 'timestep') when present, else from features column 1 (:142-156); labels via
    the class map, -1 when missing (:182-186); edges from 'txId1,txId2' or a headerless list, in
    file order, endpoints mapped to rows, unknown txIds dropped, and only same-timestep edges
    kept (:201-245).  Vectorised (pandas / numpy) instead of per-edge dict lookups.
    """
    import os

    import pandas as pd

    cls = pd.read_csv(os.path.join(data_dir, classes_csv))
    cls.columns = [c.strip() for c in cls.columns]
    if "txId" not in cls.columns:
        tx = next((c for c in cls.columns if c.lower().startswith("tx")), None)
        if tx is not None:
            cls = cls.rename(columns={tx: "txId"})
    if "time_step" in cls.columns:
        cls = cls.rename(columns={"time_step": "timestep"})
    cls_ts = "timestep" in cls.columns
    if "class" not in cls.columns:
        cc = next((c for c in cls.columns if c.lower().startswith("class")), None)
        if cc is not None:
            cls = cls.rename(columns={cc: "class"})
    cls["txId"] = pd.to_numeric(cls["txId"], errors="raise").astype(np.int64)
    cls["label"] = cls["class"].map(_label).astype(np.int64)
    keep = ["txId", "label"] + (["timestep"] if cls_ts else [])
    cls = cls[keep]
    if cls_ts:
        cls["timestep"] = pd.to_numeric(cls["timestep"], errors="raise").astype(np.int64)

    feat = pd.read_csv(os.path.join(data_dir, features_csv), header=None)
    if feat.shape[1] < 2:
        raise ValueError("features CSV appears malformed (needs at least txId + 1 column).")
    tx_ids = pd.to_numeric(feat.iloc[:, 0], errors="raise").astype(np.int64).to_numpy()
    feat_ts = _is_timestep_column(feat.iloc[:, 1])
    x = feat.iloc[:, 2:] if feat_ts else feat.iloc[:, 1:]
    x = torch.tensor(x.to_numpy(dtype=np.float32))

    nodes = pd.DataFrame({"txId": tx_ids})
    if feat_ts:
        nodes["ts_feat"] = pd.to_numeric(feat.iloc[:, 1], errors="raise").astype(np.int64).to_numpy()
    nodes = nodes.merge(cls, on="txId", how="left")  # left join: features row order
    if cls_ts:
        ts = nodes["timestep"]
    elif feat_ts:
        ts = nodes["ts_feat"]
    else:
        raise ValueError("No timestep column found in classes and features did not contain a valid timestep "
                         "column (expected classes 'time_step'/'timestep' or features column 2 in 1..49).")
    if ts.isna().any():
        raise ValueError("timestep missing for some nodes")
    y = torch.tensor(nodes["label"].fillna(-1).astype(np.int64).to_numpy())
    timestep = torch.tensor(ts.astype(np.int64).to_numpy())

    epath = os.path.join(data_dir, edgelist_csv)
    sniff = pd.read_csv(epath, nrows=5)
    header = sniff.shape[1] >= 2 and not np.issubdtype(sniff.dtypes.iloc[0], np.number)
    edges = pd.read_csv(epath, header=0 if header else None)
    if {"txId1", "txId2"}.issubset(edges.columns):
        edges = edges[["txId1", "txId2"]]
    edges = edges.iloc[:, :2].apply(pd.to_numeric, errors="coerce").dropna().astype(np.int64).to_numpy()
    # txId -> row (the last occurrence, as the reference's dict comprehension), unknown ids dropped,
    # same-timestep edges only, file order kept
    order = np.argsort(tx_ids, kind="stable")
    sorted_ids = tx_ids[order]

    def rows_of(ids):
        pos = np.searchsorted(sorted_ids, ids, side="right") - 1
        pos_c = np.maximum(pos, 0)
        ok = (pos >= 0) & (sorted_ids[pos_c] == ids) if len(sorted_ids) else np.zeros(len(ids), bool)
        return order[pos_c], ok

    src, ok_s = rows_of(edges[:, 0]) if len(edges) else (np.zeros(0, np.int64), np.zeros(0, bool))
    dst, ok_d = rows_of(edges[:, 1]) if len(edges) else (np.zeros(0, np.int64), np.zeros(0, bool))
    keep_e = ok_s & ok_d
    src, dst = src[keep_e], dst[keep_e]
    tnp = timestep.numpy()
    same = tnp[src] == tnp[dst]
    edge_index = torch.tensor(np.stack([src[same], dst[same]]).astype(np.int64))
    return GraphData(x=x, edge_index=edge_index, y=y, timestep=timestep)
