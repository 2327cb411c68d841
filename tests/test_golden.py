"""CPU: the oracle reproduces the committed golden vectors (tests/golden/make_golden.py)."""
from pathlib import Path

import numpy as np
import pytest
import torch

from oracle import pyg_ref

GOLD = Path(__file__).resolve().parent / "golden" / "elliptic600.npz"
ARCH = {"sage": dict(layers=2, heads=1), "gcn": dict(layers=2, heads=1), "gat": dict(layers=2, heads=4)}


def load(arch, z, dtype):
    return {k.split("/", 1)[1]: torch.from_numpy(z[k]).to(dtype) for k in z.files
            if k.startswith(arch + "/convs.")}


@pytest.mark.parametrize("arch", list(ARCH))
def test_oracle_reproduces_golden(arch):
    with np.load(GOLD) as z:
        x = torch.from_numpy(z["x"])
        ei = torch.from_numpy(z["edge_index"])
        out64 = pyg_ref.model_forward(arch, load(arch, z, torch.float64), x.double(), ei, **ARCH[arch])
        np.testing.assert_allclose(out64.numpy(), z[f"{arch}/logits_f64"], rtol=1e-12, atol=1e-12)
        out32 = pyg_ref.model_forward(arch, load(arch, z, torch.float32), x, ei, **ARCH[arch])
        np.testing.assert_allclose(out32.numpy(), z[f"{arch}/logits_f32"], rtol=1e-5, atol=1e-5)
        # fp32 vs fp64 truth: the 1e-5 bar is meaningful at these magnitudes
        np.testing.assert_allclose(z[f"{arch}/logits_f32"], z[f"{arch}/logits_f64"], rtol=1e-5, atol=1e-5)
        agg = pyg_ref.scatter(x.double().index_select(0, ei[0]), ei[1], x.size(0), "mean")
        np.testing.assert_allclose(agg.numpy(), z["mean_agg_f64"], rtol=1e-14, atol=1e-14)
