"""GPU: K12, the SAGEResBNNet layer tail h = dropout(relu(BatchNorm1d(z))) + r (src/models/gnn.py:182-194).

Op level against torch's own training-mode nn.BatchNorm1d (+ F.relu, the counter-hash dropout
mask of oracle/dropout_hash.py, the residual add) and autograd: outputs, running statistics,
num_batches_tracked and every gradient.  Model level: a SAGE-ResBN train step with dropout against
the CPU oracle with the same masks, and fused == unfused.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import pyg_ref
from oracle.dropout_hash import keep_mask

pytestmark = pytest.mark.gpu


def rel_l2(a, b, floor=1e-7):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).norm() / max(float(b.norm()), floor / 1e-5))


def _ref(z, r, bn_ref, p, seed):
    y = F.relu(bn_ref(z))
    if p > 0:
        m = torch.from_numpy(keep_mask(seed, z.size(0), z.size(1), p)).to(z.device)
        y = y * m / (1 - np.float32(p))
    return y + r if r is not None else y


@pytest.mark.parametrize("N,C", [(5000, 64), (777, 130), (40, 8)])
@pytest.mark.parametrize("p", [0.0, 0.2])
@pytest.mark.parametrize("momentum", [0.1, None])
@pytest.mark.parametrize("with_r", [True, False])
def test_bn_act_res_matches_torch(device, N, C, p, momentum, with_r):
    from elliptic_gnn_project_amd.fused import bn_relu_dropout_residual

    g = torch.Generator().manual_seed(N + C)
    z0 = (torch.randn(N, C, generator=g) * 2 + 0.3).to(device)
    r0 = torch.randn(N, C, generator=g).to(device) if with_r else None
    bn = torch.nn.BatchNorm1d(C, momentum=momentum).to(device)
    with torch.no_grad():
        bn.weight.copy_(torch.rand(C, generator=g) + 0.5)
        bn.bias.copy_(torch.randn(C, generator=g) * 0.1)
        bn.running_mean.copy_(torch.randn(C, generator=g))
        bn.running_var.copy_(torch.rand(C, generator=g) + 0.5)
    bn_ref = torch.nn.BatchNorm1d(C, momentum=momentum).to(device)
    bn_ref.load_state_dict(bn.state_dict())
    bn.train()
    bn_ref.train()
    seed = 1234567
    z = z0.clone().requires_grad_(True)
    r = r0.clone().requires_grad_(True) if with_r else None
    out = bn_relu_dropout_residual(z, r, bn, p, seed, None)
    zr = z0.clone().requires_grad_(True)
    rr = r0.clone().requires_grad_(True) if with_r else None
    ref = _ref(zr, rr, bn_ref, p, seed)
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(bn.running_mean, bn_ref.running_mean, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(bn.running_var, bn_ref.running_var, rtol=1e-5, atol=1e-6)
    assert int(bn.num_batches_tracked) == int(bn_ref.num_batches_tracked) == 1
    dh = torch.randn(N, C, generator=g).to(device)
    out.backward(dh)
    ref.backward(dh)
    assert rel_l2(z.grad, zr.grad) < 1e-5
    if with_r:
        assert torch.equal(r.grad, rr.grad)
    assert rel_l2(bn.weight.grad, bn_ref.weight.grad) < 1e-5
    assert rel_l2(bn.bias.grad, bn_ref.bias.grad) < 1e-5


def test_bn_stats_large_mean(device):
    """Features with a mean of ~1e3 and a spread of ~1: float64 statistics keep the variance."""
    from elliptic_gnn_project_amd.fused import bn_relu_dropout_residual

    g = torch.Generator().manual_seed(3)
    N, C = 20000, 16
    z = (1000.0 + torch.randn(N, C, generator=g, dtype=torch.float64)).float().to(device)
    bn = torch.nn.BatchNorm1d(C).to(device).train()
    out = bn_relu_dropout_residual(z, None, bn, 0.0, 0, None)
    zd = z.double()
    var = zd.var(0, unbiased=False)
    ref = F.relu((zd - zd.mean(0)) / torch.sqrt(var + 1e-5)).float()
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-4)
    unb = zd.var(0, unbiased=True)
    torch.testing.assert_close(bn.running_var.double(), 0.9 + 0.1 * unb, rtol=1e-5, atol=1e-5)


def test_bn_deterministic(device):
    from elliptic_gnn_project_amd.fused import bn_relu_dropout_residual

    g = torch.Generator().manual_seed(9)
    z0 = torch.randn(50000, 64, generator=g).to(device)
    outs = []
    for _ in range(2):
        bn = torch.nn.BatchNorm1d(64).to(device).train()
        z = z0.clone().requires_grad_(True)
        o = bn_relu_dropout_residual(z, None, bn, 0.3, 42, None)
        o.backward(torch.ones_like(o))
        outs.append((o.detach().clone(), z.grad.clone(), bn.weight.grad.clone(), bn.running_var.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("dropout", [0.0, 0.3])
def test_sage_resbn_train_step_vs_oracle(device, dropout):
    """SAGEResBNNet (sin time embedding, residual projection) train step with K12 vs the oracle
    (F.batch_norm + the same counter-hash dropout masks): logits, every gradient, running stats."""
    from elliptic_gnn_project_amd.dataset_elliptic import synthetic_elliptic
    from elliptic_gnn_project_amd.train_gnn import build_model

    data = synthetic_elliptic(num_nodes=5000, num_edges=6000, seed=8)
    ei = torch.cat([data.edge_index, data.edge_index.flip(0)], dim=1)
    x, t_idx = data.x, data.timestep
    L, H = 3, 64
    cfg = dict(arch="sage_resbn", hidden_dim=H, layers=L, dropout=dropout, use_bn=True, residual=True,
               time_embed_dim=2, time_embed_type="sin")
    torch.manual_seed(4)
    model = build_model("sage_resbn", x.size(1), cfg).to(device)
    params = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    model.train()
    torch.manual_seed(11)
    logits = model(x.to(device), ei.to(device), t_idx.to(device))
    torch.manual_seed(11)
    seeds = torch.randint(0, 2 ** 62, (L,), dtype=torch.int64).tolist()
    N = x.size(0)
    masks = [torch.from_numpy(keep_mask(seeds[l], N, H, dropout)) for l in range(L - 1)] if dropout > 0 else None
    mask = data.y >= 0
    cw = pyg_ref.class_weight(data.y[mask])
    loss = pyg_ref.ce_loss(logits[mask.to(device)], data.y[mask].to(device), cw.to(device))
    loss.backward()
    bn_state = {k: v.clone() for k, v in params.items() if "running" in k}
    kw = dict(layers=L, dropout=dropout, training=True, dropout_masks=masks, t_idx=t_idx, time_embed_dim=2,
              time_embed_type="sin", max_timestep=49)
    ref = pyg_ref.model_forward("sage_resbn", params, x, ei, bn_state=bn_state, **kw)
    torch.testing.assert_close(logits.detach().cpu(), ref, rtol=1e-5, atol=1e-5)
    for k in bn_state:  # the oracle's F.batch_norm updated its copies in place
        torch.testing.assert_close(model.state_dict()[k].cpu(), bn_state[k], rtol=1e-5, atol=1e-6)
    _, grads = pyg_ref.train_step_grads("sage_resbn", params, x, ei, data.y, mask, cw,
                                        bn_state={k: v.clone() for k, v in params.items() if "running" in k}, **kw)
    for k, v in model.named_parameters():
        assert rel_l2(v.grad, grads[k]) < 1e-5, k


def test_sage_resbn_fused_equals_unfused(device):
    from elliptic_gnn_project_amd.dataset_elliptic import synthetic_elliptic
    from elliptic_gnn_project_amd.train_gnn import build_model

    data = synthetic_elliptic(num_nodes=4000, num_edges=5000, seed=12)
    ei = torch.cat([data.edge_index, data.edge_index.flip(0)], dim=1).to(device)
    x, t_idx = data.x.to(device), data.timestep.to(device)
    cfg = dict(arch="sage_resbn", hidden_dim=64, layers=3, dropout=0.0, use_bn=True, residual=True,
               time_embed_dim=2, time_embed_type="sin")
    res = []
    for fused in (True, False):
        torch.manual_seed(4)
        model = build_model("sage_resbn", x.size(1), cfg).to(device).train()
        model.fused_bn = fused
        out = model(x, ei, t_idx)
        out.square().sum().backward()
        res.append((out.detach(), {k: v.grad.clone() for k, v in model.named_parameters()},
                    {k: v.clone() for k, v in model.state_dict().items() if "running" in k}))
    torch.testing.assert_close(res[0][0], res[1][0], rtol=1e-5, atol=1e-5)
    for k in res[0][1]:
        a, b = res[0][1][k], res[1][1][k]
        if k.endswith("lin_l.bias") and not k.startswith("convs.2"):
            # a conv bias feeding BatchNorm has an exactly-zero gradient: both are rounding noise;
            # compare it on the scale of its conv's weight gradient
            scale = float(res[1][1][k.replace("bias", "weight")].norm())
            assert float((a - b).norm()) <= 1e-5 * scale, k
            continue
        assert rel_l2(a, b) < 1e-5, k
    for k in res[0][2]:
        torch.testing.assert_close(res[0][2][k], res[1][2][k], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("dim,T", [(2, 50), (5, 50), (8, 1)])
@pytest.mark.parametrize("Fin", [165, 166, 300])
def test_time_inject_sin_matches_torch(device, dim, T, Fin):
    """K13 vs SAGEResBNNet's torch path (_sinusoid + cat), including out-of-range timesteps."""
    from elliptic_gnn_project_amd.fused import time_inject_sin
    from elliptic_gnn_project_amd.gnn import SAGEResBNNet

    g = torch.Generator().manual_seed(dim)
    N = 3001
    x = torch.randn(N, Fin, generator=g).to(device)
    t = torch.randint(-2, 60, (N,), generator=g).to(device)
    m = SAGEResBNNet(Fin, 16, layers=2, time_embed_dim=dim, time_embed_type="sin", max_timestep=T).to(device)
    ref = torch.cat([x, m._sinusoid(t)], dim=1)
    out = time_inject_sin(x, t, dim, T)
    torch.testing.assert_close(out, ref, rtol=1e-6, atol=1e-6)
    assert torch.equal(out[:, :Fin], x)
    assert torch.equal(m._inject_time(x, t), out)


def test_time_inject_cached_for_registered_input(device):
    """K13's [x | sin(t)] is a function of constants for a registered x: computed once, cached on
    x, registered itself (layer 1's GEMMs read its image); an in-place edit of x recomputes it."""
    from elliptic_gnn_project_amd.fused import time_inject_sin
    from elliptic_gnn_project_amd.planes import is_registered, register_input

    g = torch.Generator().manual_seed(5)
    x = register_input(torch.randn(3000, 165, generator=g).to(device))
    t = torch.randint(1, 50, (3000,), generator=g).to(device)
    a = time_inject_sin(x, t, 2, 49)
    b = time_inject_sin(x, t, 2, 49)
    assert a is b and is_registered(a)
    x.mul_(2.0)
    c = time_inject_sin(x, t, 2, 49)
    assert c is not a
    torch.testing.assert_close(c[:, :165], x)
    u = torch.randn(100, 165, generator=g).to(device)  # unregistered: no cache, fresh each call
    assert time_inject_sin(u, t[:100], 2, 49) is not time_inject_sin(u, t[:100], 2, 49)
