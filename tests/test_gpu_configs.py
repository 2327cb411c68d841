"""GPU parity for the model shapes the reference's shipped configs train, beyond the BASELINE
presets (VERDICT r4 missing #5): one train step (fwd + masked CE + bwd) against the float64
oracle with the very same dropout masks, logits rtol = atol = 1e-5 and every parameter gradient
relative L2 <= 1e-5, on a 5,000-node Elliptic-shaped graph, registered (x declared constant, as
train_gnn.main / bench.py do) and unregistered; the largest shape also at the full 203,769 nodes.

    sage_resbn_k14   /root/reference/configs/sage_resbn_k14.yaml:9-21   SAGE-ResBN 3L/128, learned
                     time embedding dim 8 (time_embed_type defaults to 'learned',
                     src/train_gnn.py:100), in 165 + 8 = 173
    resbn_k8_sin2    /root/reference/configs/sage_resbn_k8_sin2.yaml    SAGE-ResBN 3L/64 + sin 2
    rec_k9           /root/reference/configs/rec_k9.yaml:10-13,36-38    (same shape, window 9)
    sage_l3          /root/reference/configs/sage_l3_k{6,10,14,18}.yaml SAGE 3L/128, dropout 0.3/0.4,
                     time scalar (in 166)
    *_h256           hidden_dim 256 (any width build_model accepts, src/train_gnn.py:67-104): the
                     convs' GEMMs past the split-bf16 kernels' 128-column envelope

(The shipped configs set amp: true; the fused steps run fp32 under autocast — custom_fwd casts
their inputs — which test_gpu_train_main.py covers; here the step runs fp32 directly.)
"""
import pytest
import torch

import relu_ties
from oracle import pyg_ref
from oracle.dropout_hash import keep_mask

pytestmark = pytest.mark.gpu

SHAPES = {
    "sage_resbn_k14": dict(arch="sage_resbn", hidden_dim=128, layers=3, dropout=0.2, time_embed_dim=8,
                           time_embed_type="learned", max_timestep=49, use_time_scalar=False, train_window_k=14),
    "resbn_k8_sin2": dict(arch="sage_resbn", hidden_dim=64, layers=3, dropout=0.2, time_embed_dim=2,
                          time_embed_type="sin", max_timestep=49, use_time_scalar=False, train_window_k=8),
    "rec_k9": dict(arch="sage_resbn", hidden_dim=64, layers=3, dropout=0.2, time_embed_dim=2,
                   time_embed_type="sin", max_timestep=49, use_time_scalar=False, train_window_k=9),
    "sage_l3_k18": dict(arch="sage", hidden_dim=128, layers=3, dropout=0.4, use_time_scalar=True,
                        train_window_k=18),
    # past the split-bf16 GEMMs' envelope (out > 128): linear._TiledLinear — exact-f32 MFMA NT,
    # blocked TN — not torch's F.linear; dropout 0: the per-conv path
    "sage_h256": dict(arch="sage", hidden_dim=256, layers=2, dropout=0.0, use_time_scalar=True,
                      train_window_k=10),
    "gcn_h256": dict(arch="gcn", hidden_dim=256, layers=2, dropout=0.0, use_time_scalar=True,
                     train_window_k=10),
    "gat_h256": dict(arch="gat", hidden_dim=256, heads=4, layers=2, dropout=0.0, use_time_scalar=True,
                     train_window_k=10),
}


def rel_l2(a, b, floor=1e-30):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).norm() / max(float(b.norm()), floor))


def _data(cfg, n, e):
    from elliptic_gnn_project_amd.dataset_elliptic import prepare_inputs, synthetic_elliptic

    return prepare_inputs(synthetic_elliptic(num_nodes=n, num_edges=e, seed=42),
                          dict(use_time_scalar=cfg["use_time_scalar"], symmetrize_edges=True,
                               train_window_k=cfg["train_window_k"]))


def _step_vs_oracle(device, cfg, data, registered):
    from elliptic_gnn_project_amd.planes import register_input
    from elliptic_gnn_project_amd.train_gnn import build_model

    L, H, p = cfg["layers"], cfg["hidden_dim"], cfg["dropout"]
    te = cfg.get("time_embed_dim", 0)
    N = data.x.size(0)
    torch.manual_seed(4)
    model = build_model(cfg["arch"], data.x.size(1), cfg).to(device)
    params = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    model.train()
    xd = data.x.to(device)
    if registered:
        register_input(xd)
    t_idx = data.timestep.to(device) if te else None
    bn = cfg["arch"] == "sage_resbn"
    zs, hooks = relu_ties.capture_hidden_z(model) if bn else ([], [])
    torch.manual_seed(11)
    logits = model(xd, data.edge_index.to(device), t_idx)
    for hk in hooks:
        hk.remove()
    torch.manual_seed(11)
    seeds = torch.randint(0, 2 ** 62, (L,), dtype=torch.int64).tolist()
    masks = [torch.from_numpy(keep_mask(seeds[l], N, H, p)) for l in range(L - 1)]
    tm = data.train_mask
    cw = pyg_ref.class_weight(data.y[tm])
    loss = pyg_ref.ce_loss(logits[tm.to(device)], data.y[tm].to(device), cw.to(device))
    loss.backward()
    p64 = {k: v.double() if v.is_floating_point() else v for k, v in params.items()}
    kw = dict(layers=L, dropout=p, training=True, dropout_masks=masks)
    if te:
        kw.update(t_idx=data.timestep, time_embed_dim=te, time_embed_type=cfg["time_embed_type"],
                  max_timestep=cfg["max_timestep"])
    bn_state = {k: v.clone() for k, v in p64.items() if "running" in k} if bn else None
    x64 = data.x.double()
    trace = []
    ref = pyg_ref.model_forward(cfg["arch"], p64, x64, data.edge_index, bn_state=bn_state, trace=trace, **kw)
    torch.testing.assert_close(logits.detach().cpu().double(), ref, rtol=1e-5, atol=1e-5)
    force = None
    if bn:
        for k in bn_state:  # the running statistics K12 updated, vs F.batch_norm's in-place update
            torch.testing.assert_close(model.state_dict()[k].cpu().double(), bn_state[k], rtol=1e-5, atol=1e-6)
        force = relu_ties.relu_force(zs, p64, trace)  # the device's resolution of ReLU ties (relu_ties.py)
        assert sum(int(v[0].numel()) for v in force.values()) <= 8, force
    ref_loss, grads = pyg_ref.train_step_grads(
        cfg["arch"], p64, x64, data.edge_index, data.y, tm, cw.double(),
        bn_state={k: v.clone() for k, v in p64.items() if "running" in k} if bn else None, relu_force=force, **kw)
    assert abs(float(loss.detach()) - float(ref_loss)) <= 1e-5 * max(1.0, abs(float(ref_loss)))
    if te and cfg["time_embed_type"] == "learned":
        assert "time_emb.weight" in grads  # the learned embedding is trained through the step
    for k, v in model.named_parameters():
        # a hidden conv's bias feeds BatchNorm: its true gradient is zero; the output bias gradient
        # is Σ dlogits over the train rows, which the class weights balance toward zero (on 5,000
        # nodes |Σ| ~ 1e-2 of Σ|.|): both are held to 1e-7 absolute (floor 1e-2), not relative
        conv_bias = k.startswith("convs.") and k.endswith("lin_l.bias")
        zero = conv_bias and (bn or int(k.split(".")[1]) == L - 1)
        e = rel_l2(v.grad, grads[k], floor=1e-2 if zero else 1e-30)
        assert e < 1e-5, (k, e)


@pytest.mark.parametrize("registered", [True, False])
@pytest.mark.parametrize("shape", list(SHAPES))
def test_shipped_config_train_step(device, shape, registered):
    cfg = SHAPES[shape]
    _step_vs_oracle(device, cfg, _data(cfg, 5000, 6000), registered)


@pytest.mark.parametrize("registered", [True, False])
def test_sage_resbn_k14_full_size(device, registered):
    """sage_resbn_k14 (the widest shipped ResBN: hidden 128, in 173) on the full 203,769-node
    graph: K12's statistics over every row block and the F = 128 gathers at the real hub degrees."""
    cfg = SHAPES["sage_resbn_k14"]
    _step_vs_oracle(device, cfg, _data(cfg, 203_769, 234_355), registered)
