"""Host-side pieces of train_gnn.main, CPU only: the per-timestep PR-AUC tail of metrics.json
(src/train_gnn.py:497-519), the hub-ablation edge filter (:526-539), RunLogger's CSV
(src/utils/logger.py:5-27), the masked-CE empty-selection rule and the loss divisor fields."""
import numpy as np
import torch

from elliptic_gnn_project_amd import metrics as M
from elliptic_gnn_project_amd.dataset_elliptic import prepare_inputs, synthetic_elliptic
from elliptic_gnn_project_amd.train_gnn import RunLogger, hub_edge_mask, per_timestep_pr_auc


def test_per_timestep_pr_auc_known_answer():
    ts = np.array([44, 44, 45, 45, 46, 46, 47, 47, 48, 48, 49, 49])
    y = np.array([1, 0, 0, 1, 1, 0, 0, 1, 1, 0, 1, 0])
    p = np.array([0.9, 0.1, 0.8, 0.2, 0.6, 0.4, 0.3, 0.7, 0.55, 0.45, 0.2, 0.9])
    out = per_timestep_pr_auc(y, p, ts)
    # two nodes per timestep: AP = 1 when the positive ranks first, 0.5 otherwise
    assert out["test_pr_auc_by_time"] == [1.0, 0.5, 1.0, 1.0, 1.0, 0.5]
    assert out["pr_auc_last1"] == 0.5
    assert abs(out["pr_auc_last3"] - 2.5 / 3) < 1e-12
    assert abs(out["pr_auc_last5"] - 4.0 / 5) < 1e-12
    assert per_timestep_pr_auc(y[:4], p[:4], ts[:4]) == {"test_pr_auc_by_time": [1.0, 0.5], "pr_auc_last1": 0.5}
    assert per_timestep_pr_auc(y[:0], p[:0], ts[:0]) == {}


def test_hub_edge_mask_matches_definition():
    g = torch.Generator().manual_seed(0)
    N = 200
    ei = torch.randint(0, N, (2, 1000), generator=g)
    hubs, keep, nh = hub_edge_mask(ei, N, 0.05)
    assert nh == 10 and int(hubs.sum()) == 10
    deg = np.bincount(ei[0].numpy(), minlength=N) + np.bincount(ei[1].numpy(), minlength=N)
    # every hub's degree >= every non-hub's (top-k), and an edge survives iff neither end is a hub
    assert deg[hubs.numpy()].min() >= deg[~hubs.numpy()].max()
    h = hubs.numpy()
    want = ~(h[ei[0].numpy()] | h[ei[1].numpy()])
    assert np.array_equal(keep.numpy(), want)
    _, keep0, nh0 = hub_edge_mask(ei, N, 0.0)
    assert nh0 == 0 and bool(keep0.all())


def test_run_logger_csv(tmp_path):
    lg = RunLogger(str(tmp_path))
    lg.log_epoch(1, 0.5, 0.25)
    lg.log_epoch(2, 0.25, 0.5)
    lg.close()
    assert (tmp_path / "training_log.csv").read_text().splitlines() == [
        "epoch,train_loss,val_pr_auc", "1,0.500000,0.250000", "2,0.250000,0.500000"]


def test_prepare_inputs_caches_split_counts():
    d = prepare_inputs(synthetic_elliptic(num_nodes=2000, num_edges=3000, seed=1),
                       dict(use_time_scalar=True, symmetrize_edges=True, train_window_k=10))
    assert d.n_train == int(d.train_mask.sum()) and d.n_val == int(d.val_mask.sum())
    assert d.to("cpu").n_train == d.n_train  # plain ints travel with .to()


def test_metric_names_are_the_reference_ones():
    y = np.array([0, 1, 1, 0, 1])
    p = np.array([0.1, 0.8, 0.6, 0.3, 0.2])
    assert M.pick_threshold_max_f1(y, p)[0] in set(p.tolist()) | {1.0}
