"""CSV -> PyG-free graph file (the reference's src/data/build_graph.py:6-31).

    python -m elliptic_gnn_project_amd.build_graph --config configs/split.yaml

Loads the Elliptic CSVs (dataset_elliptic.load_elliptic_csv), builds the temporal masks
(t_train_end / t_val_end) and writes ``<processed_dir>/graph.npz`` (plain arrays, loadable with
allow_pickle=False — the reference's pickled PyG ``graph.pt`` needs torch_geometric to load)
plus ``meta.json`` with the node / edge / feature / label counts.
"""
from __future__ import annotations

import argparse
import json
import os

import yaml

from .dataset_elliptic import load_elliptic_csv, make_temporal_masks, save_graph


def main(cfg: dict) -> str:
    g = load_elliptic_csv(cfg["data_dir"], cfg.get("features_csv", "elliptic_txs_features.csv"),
                          cfg.get("classes_csv", "elliptic_txs_classes.csv"),
                          cfg.get("edgelist_csv", "elliptic_txs_edgelist.csv"))
    make_temporal_masks(g, cfg["t_train_end"], cfg["t_val_end"])
    out_dir = cfg["processed_dir"]
    os.makedirs(out_dir, exist_ok=True)
    path = os.path.join(out_dir, "graph.npz")
    save_graph(path, g)
    meta = {"num_nodes": int(g.x.size(0)), "num_edges": int(g.edge_index.size(1)),
            "num_features": int(g.x.size(1)),
            "label_counts": {str(v): int((g.y == v).sum()) for v in (-1, 0, 1)}, "graph_file": path}
    with open(os.path.join(out_dir, "meta.json"), "w") as fh:
        json.dump(meta, fh, indent=2)
    print(f"Saved graph to {path}")
    return path


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", required=True)
    a = ap.parse_args()
    with open(a.config) as fh:
        main(yaml.safe_load(fh))
