"""The loss variants against vectors from the REFERENCE's own ``_make_loss_fn`` / ``class_weight``
(src/train_gnn.py:116-183; tests/golden/make_loss_golden.py): class-weighted CE, focal (gamma 1,
2), time weighting (linear, sqrt, the 1e-3 clamp) and the time-embedding L2 — loss and gradients.
CPU here; the GPU copy runs the same cases on the device (and the plain case through the fused
masked-CE kernel)."""
import os

import numpy as np
import pytest
import torch

from elliptic_gnn_project_amd.train_gnn import _make_loss_fn, class_weight

GOLD = os.path.join(os.path.dirname(__file__), "golden", "loss_golden.npz")
CASES = {
    "ce_weighted": (dict(), False),
    "focal_g1": (dict(focal_loss=True, focal_gamma=1.0), False),
    "focal_g2": (dict(focal_loss=True, focal_gamma=2.0), False),
    "time_linear": (dict(time_loss_weighting="linear"), False),
    "time_sqrt": (dict(time_loss_weighting="sqrt"), False),
    "focal_time_sqrt": (dict(focal_loss=True, focal_gamma=2.0, time_loss_weighting="sqrt"), False),
    "embed_l2": (dict(time_embed_l2=0.01), True),
    "time_linear_embed_l2": (dict(time_loss_weighting="linear", time_embed_l2=0.05), True),
}


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD)


class _TimeModel(torch.nn.Module):
    def __init__(self, emb):
        super().__init__()
        self.time_embed_dim = 4 if emb is not None else 0
        self.time_emb = None
        if emb is not None:
            self.time_emb = torch.nn.Embedding(*emb.shape)
            with torch.no_grad():
                self.time_emb.weight.copy_(torch.from_numpy(emb))


def _run_case(gold, name, device):
    cfg, with_emb = CASES[name]
    t_min, t_max = (int(v) for v in gold["t_range"])
    model = _TimeModel(gold[f"{name}/emb"] if with_emb else None).to(device)
    cw = torch.from_numpy(gold["class_weight"])
    fn = _make_loss_fn(cfg, cw, model, t_min, t_max)
    lg = torch.from_numpy(gold["logits"]).to(device).requires_grad_(True)
    y = torch.from_numpy(gold["y"]).to(device)
    t = torch.from_numpy(gold["t_idx"]).to(device)
    loss = fn(lg, y, t)
    loss.backward()
    return loss, lg.grad, (model.time_emb.weight.grad if with_emb else None)


def test_class_weight_matches_reference(gold):
    y = torch.from_numpy(gold["y"])
    np.testing.assert_array_equal(class_weight(y).numpy(), gold["class_weight"])
    np.testing.assert_array_equal(class_weight(torch.ones(7, dtype=torch.long)).numpy(), gold["class_weight_allpos"])


@pytest.mark.parametrize("name", sorted(CASES))
def test_loss_variant_matches_reference(gold, name):
    loss, dl, demb = _run_case(gold, name, "cpu")
    np.testing.assert_allclose(loss.item(), float(gold[f"{name}/loss"]), rtol=1e-6, atol=0)
    np.testing.assert_allclose(dl.numpy(), gold[f"{name}/dlogits"], rtol=1e-5, atol=1e-9)
    if demb is not None:
        np.testing.assert_allclose(demb.numpy(), gold[f"{name}/demb"], rtol=1e-5, atol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
def test_loss_variant_matches_reference_gpu(gold, name, device):
    loss, dl, demb = _run_case(gold, name, device)
    np.testing.assert_allclose(loss.item(), float(gold[f"{name}/loss"]), rtol=1e-5, atol=0)
    np.testing.assert_allclose(dl.cpu().numpy(), gold[f"{name}/dlogits"], rtol=1e-5, atol=1e-8)
    if demb is not None:
        np.testing.assert_allclose(demb.cpu().numpy(), gold[f"{name}/demb"], rtol=1e-5, atol=1e-10)


@pytest.mark.gpu
def test_fused_masked_ce_matches_reference(gold, device):
    """The default configuration's fused kernel (loss_fn.full -> K8) on the same rows."""
    cw = torch.from_numpy(gold["class_weight"])
    fn = _make_loss_fn({}, cw, torch.nn.Module(), 1, 34)
    assert fn.plain
    n = gold["logits"].shape[0]
    # the golden rows scattered into a larger logit matrix, masked rows elsewhere
    N = 3 * n
    rows = torch.arange(0, N, 3)
    logits = torch.randn(N, 2)
    logits[rows] = torch.from_numpy(gold["logits"])
    y = torch.full((N,), -1, dtype=torch.long)
    y[rows] = torch.from_numpy(gold["y"])
    mask = torch.zeros(N, dtype=torch.bool)
    mask[rows] = True
    lg = logits.to(device).requires_grad_(True)
    loss = fn.full(lg, y.to(device), mask.to(device))
    loss.backward()
    np.testing.assert_allclose(loss.item(), float(gold["ce_weighted/loss"]), rtol=1e-6, atol=0)
    g = lg.grad.cpu()
    np.testing.assert_allclose(g[rows].numpy(), gold["ce_weighted/dlogits"], rtol=1e-5, atol=1e-9)
    assert not g[~mask].any()
