"""GPU end to end: train_gnn.main (src/train_gnn.py:282-564) on a seeded synthetic graph.

Checks the artefact set the reference's analysis scripts read (scores/labels/node ids/
timesteps per split, best.ckpt, metrics.json with the per-timestep PR-AUC tail,
metrics_hub_removed.json, training_log.csv, config_used.yaml) and that metrics.json is the
metrics of the saved test scores (src/utils/metrics.py restated, golden-pinned elsewhere).
"""
import json

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _cfg(tmp_path, arch, **kw):
    base = dict(run_name=f"e2e_{arch}", output_root=str(tmp_path), arch=arch, hidden_dim=32, layers=2, heads=4,
                dropout=0.2, lr=0.005, weight_decay=1e-4, max_epochs=4, patience=10, grad_clip=1.0, amp=False,
                symmetrize_edges=True, use_time_scalar=True, train_window_k=10, calibrate_temperature=True,
                ablate_hubs_frac=0.02, topk=50, synthetic=dict(num_nodes=8000, num_edges=12000, seed=5))
    base.update(kw)
    return base


@pytest.mark.parametrize("arch", ["sage", "gcn", "gat", "sage_resbn"])
def test_main_artefacts(device, tmp_path, arch):
    from elliptic_gnn_project_amd import metrics as M
    from elliptic_gnn_project_amd.train_gnn import main

    extra = dict(time_embed_dim=2, time_embed_type="learned", use_time_scalar=False, layers=3, time_embed_l2=1e-3,
                 time_loss_weighting="sqrt") if arch == "sage_resbn" else {}
    cfg = _cfg(tmp_path, arch, **extra)
    metrics = main(cfg)
    out = tmp_path / "gnn" / cfg["run_name"]
    for f in ("scores_val.npy", "scores_test.npy", "y_val.npy", "y_test.npy", "node_idx_val.npy", "node_idx_test.npy",
              "timestep_val.npy", "timestep_test.npy", "best.ckpt", "metrics.json", "metrics_hub_removed.json",
              "training_log.csv", "config_used.yaml"):
        assert (out / f).exists(), f
    m = json.loads((out / "metrics.json").read_text())
    p_te = np.load(out / "scores_test.npy")
    y_te = np.load(out / "y_test.npy")
    ts = np.load(out / "timestep_test.npy")
    yb = (y_te == 1).astype(int)
    assert m["pr_auc_illicit"] == pytest.approx(M.pr_auc_illicit(yb, p_te), abs=1e-12)
    assert m["n_test"] == len(y_te)
    # per-timestep PR-AUC (src/train_gnn.py:497-519)
    uniq = sorted(set(ts.tolist()))
    by_t = [M.pr_auc_illicit((y_te[ts == t] == 1).astype(int), p_te[ts == t]) for t in uniq]
    np.testing.assert_allclose(m["test_pr_auc_by_time"], by_t, rtol=0, atol=1e-12, equal_nan=True)
    assert m["pr_auc_last1"] == pytest.approx(by_t[-1], nan_ok=True)
    assert m["pr_auc_last3"] == pytest.approx(sum(by_t[-3:]) / 3, nan_ok=True)
    assert m["pr_auc_last5"] == pytest.approx(sum(by_t[-5:]) / 5, nan_ok=True)
    h = json.loads((out / "metrics_hub_removed.json").read_text())
    assert h["n_hubs"] == int(0.02 * 8000) and h["hub_fraction"] == 0.02 and h["threshold"] == m["threshold"]
    log = (out / "training_log.csv").read_text().strip().splitlines()
    assert log[0] == "epoch,train_loss,val_pr_auc" and len(log) == 1 + 4
    state = torch.load(out / "best.ckpt", weights_only=True)
    assert any(k.startswith("convs.0.") for k in state)
    assert metrics["best_val_pr_auc"] == m["best_val_pr_auc"]


def test_make_optimizer_many_tensors_falls_back(device):
    """ClipAdam holds <= ADAM_MAX_TENSORS tensors; a 6-layer SAGE-ResBN with a learned
    time embedding has more, and must train (torch Adam + clip_grad_norm_) instead of raising."""
    from elliptic_gnn_project_amd import _lib
    from elliptic_gnn_project_amd.train_gnn import build_model, make_optimizer
    from elliptic_gnn_project_amd.train_ops import ClipAdam

    cfg = dict(hidden_dim=16, layers=6, dropout=0.1, time_embed_dim=2, time_embed_type="learned", lr=1e-3,
               weight_decay=0.0, grad_clip=1.0)
    model = build_model("sage_resbn", 20, cfg).to(device)
    assert len(list(model.parameters())) > _lib.ADAM_MAX_TENSORS
    opt = make_optimizer(model, cfg, device, use_amp=False)
    assert not isinstance(opt, ClipAdam)
    small = build_model("sage", 20, dict(hidden_dim=16, layers=2, dropout=0.1)).to(device)
    assert isinstance(make_optimizer(small, dict(cfg), device, use_amp=False), ClipAdam)


def test_amp_config_runs_the_fused_step(device, tmp_path, monkeypatch):
    """configs/sage.yaml keeps the reference's amp: true (src/train_gnn.py:291-292).  On the fp32
    fused SAGENet that is the fused step (ClipAdam with GradScaler's non-finite skip, the fused
    masked CE) and it trains exactly as amp: false: identical losses and best weights after 3 epochs."""
    from pathlib import Path

    import yaml

    from elliptic_gnn_project_amd import train_gnn, train_ops
    from elliptic_gnn_project_amd.train_ops import ClipAdam

    base = yaml.safe_load((Path(__file__).resolve().parents[1] / "configs" / "sage.yaml").read_text())
    assert base["amp"] is True
    opts, ce_calls = {}, []
    make = train_gnn.make_optimizer
    ce = train_ops.masked_cross_entropy

    def spy_make(model, cfg, dev, use_amp):
        opts[use_amp] = make(model, cfg, dev, use_amp)
        return opts[use_amp]

    def spy_ce(*a, **k):
        ce_calls.append(1)
        return ce(*a, **k)

    monkeypatch.setattr(train_gnn, "make_optimizer", spy_make)
    monkeypatch.setattr(train_ops, "masked_cross_entropy", spy_ce)
    res = {}
    for amp in (True, False):
        cfg = dict(base, amp=amp, run_name=f"amp_{amp}", output_root=str(tmp_path), max_epochs=3, patience=10,
                   processed_dir=str(tmp_path / "none"), synthetic=dict(num_nodes=6000, num_edges=9000, seed=3))
        n0 = len(ce_calls)
        train_gnn.main(cfg)
        assert len(ce_calls) - n0 == 3, "the fused masked CE ran every epoch"
        out = tmp_path / "gnn" / cfg["run_name"]
        res[amp] = ((out / "training_log.csv").read_text(), torch.load(out / "best.ckpt", weights_only=True))
    assert isinstance(opts[True], ClipAdam) and opts[True].skip_nonfinite
    assert isinstance(opts[False], ClipAdam) and not opts[False].skip_nonfinite
    assert res[True][0] == res[False][0]
    for k, v in res[True][1].items():
        assert torch.equal(v, res[False][1][k]), k


def test_clip_adam_skips_nonfinite_update(device):
    """GradScaler.step semantics of ClipAdam(skip_nonfinite): an inf gradient leaves parameters,
    moments and the step count untouched; the next finite step proceeds as step 1."""
    from elliptic_gnn_project_amd.train_ops import ClipAdam

    torch.manual_seed(0)
    p = torch.nn.Parameter(torch.randn(100, device=device))
    q = torch.nn.Parameter(p.detach().clone())
    a = ClipAdam([p], lr=0.01, max_norm=1.0, skip_nonfinite=True)
    b = ClipAdam([q], lr=0.01, max_norm=1.0)
    g = torch.randn(100, device=device)
    p.grad = g.clone()
    p.grad[7] = float("inf")
    before = p.detach().clone()
    a.step()
    torch.cuda.synchronize()
    assert torch.equal(p.detach(), before) and float(a.param_groups[0]["step_t"]) == 0.0
    p.grad = g.clone()
    q.grad = g.clone()
    a.step()
    b.step()
    assert torch.equal(p.detach(), q.detach())
    assert float(a.param_groups[0]["step_t"]) == 1.0
