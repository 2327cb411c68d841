"""GPU: the f32 transposed mean (gnn_aggregate_f32 MEAN_BWD — SAGEConv's mean backward, PyG's
``grad / count`` per element) keeps the exact IEEE division.  Only the bf16-storage path
(configs[4]) multiplies by one correctly rounded reciprocal per slot (DESIGN.md §4 bf16 storage,
INTEGRATION.md); this pins the f32 path so it cannot drift onto the reciprocal.

Graph: every source node has exactly ONE out-edge, so each output row is a single quotient
dout[i] / max(deg[i], 1) with no summation order involved — it must equal torch's correctly
rounded division bit for bit, for every width class of the gather (narrow F <= 4, lane groups,
wave-wide)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("F", [1, 2, 4, 16, 64, 128, 166])
def test_f32_mean_bwd_is_the_exact_division(device, F):
    from elliptic_gnn_project_amd import _lib
    from elliptic_gnn_project_amd.aggregation import aggregate
    from elliptic_gnn_project_amd.graph import get_plan

    N = 50_000
    g = torch.Generator().manual_seed(F)
    src = torch.arange(N)
    # skewed targets: in-degrees from 0 to a few hundred (hub rows: the split / cooperative paths)
    dst = (torch.rand(N, generator=g) ** 3 * N).long().clamp_(max=N - 1)
    ei = torch.stack([src, dst]).to(device)
    plan = get_plan(ei, N, _lib.LOOPS_KEEP)
    dout = (torch.randn(N, F, generator=g) * torch.exp(torch.randn(N, 1, generator=g) * 3)).to(device)
    y = aggregate(plan, dout, _lib.AGG_MEAN_BWD, transpose=True, nodew=plan.deg)
    deg = plan.deg.clamp(min=1.0)
    ref = dout[dst.to(device)] / deg[dst.to(device)].view(N, 1)  # row j: its one edge j -> dst[j]
    assert int(plan.deg.max()) > 32  # hub targets present
    assert torch.equal(y, ref)
