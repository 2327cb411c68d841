"""ReLU ties in the SAGE-ResBN parity tests (test infrastructure, not a test module).

A hidden layer's ReLU acts on BN(z); where |BN(z)| is at the level of z's fp32 rounding (a few
elements of 13 M at full size), the device and the float64 oracle may decide the ReLU either way.
The forward is continuous there (relu(0) = 0), but the gradient takes a different path through
such an element, so a strict gradient comparison would test the tie-break, not the kernels.
These helpers read the device's decision from its own conv outputs (forward hooks on the hidden
convs, the BN batch statistics re-derived in float64) and hand the oracle exactly those
decisions for the near-tie elements (oracle/pyg_ref.py model_forward relu_force); everywhere
else the oracle's own ReLU stands."""
import torch


def capture_hidden_z(model):
    """Forward hooks recording each hidden conv's output z (the input of BN / K12)."""
    zs = []
    hooks = [c.register_forward_hook(lambda m, i, o: zs.append(o.detach().float().cpu())) for c in model.convs[:-1]]
    return zs, hooks


def relu_force(zs_gpu, params, trace, eps=1e-5, window=1e-5):
    """{layer: (flat indices, device decision)} for the elements whose oracle BN output lies within
    ``window`` of zero and whose device decision differs from the oracle's."""
    force = {}
    for l, (zg, zo) in enumerate(zip(zs_gpu, trace)):
        z = zg.double()
        mean, var = z.mean(0), z.var(0, unbiased=False)
        y = (z - mean) / torch.sqrt(var + eps) * params[f"bns.{l}.weight"].double() + params[f"bns.{l}.bias"].double()
        dec = (y > 0).flatten()
        cand = ((zo.abs() < window).flatten() & (dec != (zo > 0).flatten())).nonzero().flatten()
        if cand.numel():
            force[l] = (cand, dec[cand])
    return force
