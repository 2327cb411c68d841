"""INTEGRATION.md §B is executable: its ctypes binding (gnn_graph mirroring include/gnnmp.h,
csr_split/csc_split included) is extracted verbatim, run, and its sage_mean compared with the
oracle's PyG scatter-mean on graphs with isolated nodes, duplicates, self loops and a hub."""
import os
import re

import pytest
import torch

from oracle import pyg_ref

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _snippet():
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = doc[doc.index("## B."):]
    return re.search(r"```python\n(.*?)```", sec, re.S).group(1)


def test_section_b_struct_mirrors_header():
    src = _snippet()
    hdr = open(os.path.join(ROOT, "include", "gnnmp.h")).read()
    body = hdr[hdr.index("typedef struct {\n  int64_t num_nodes;"):]
    body = body[: body.index("} gnn_graph;")]
    fields = re.findall(r"\*?\s*(\w+);", body)
    doc_fields = re.findall(r'\("(\w+)", ctypes\.', src[src.index("class gnn_graph"):src.index("def build_plan")])
    assert doc_fields == fields


@pytest.mark.gpu
@pytest.mark.parametrize("n,e,seed,hub", [(50, 20, 1, None), (4000, 12000, 2, None), (300, 600, 3, 7)])
def test_section_b_runs_verbatim(device, n, e, seed, hub):
    ns = {}
    cwd = os.getcwd()
    os.chdir(ROOT)  # the snippet loads the library by its in-tree path
    try:
        exec(compile(_snippet(), "INTEGRATION.md#B", "exec"), ns)
    finally:
        os.chdir(cwd)
    g = torch.Generator().manual_seed(seed)
    src = torch.randint(0, n, (e,), generator=g)
    dst = torch.randint(0, n, (e,), generator=g)
    if hub is not None:
        src = torch.cat([src, torch.randint(0, n, (3000,), generator=g), torch.arange(5)])
        dst = torch.cat([dst, torch.full((3000,), hub), torch.arange(5)])  # hub + 5 self loops
    src = torch.cat([src, src[:7]])
    dst = torch.cat([dst, dst[:7]])  # duplicates
    ei = torch.stack([src, dst]).long()
    x = torch.randn(n, 166, generator=g)
    eid = ei.to(device)
    plan, keep = ns["build_plan"](eid, n)
    deg = ns["in_degree"](plan, n, device)
    out = ns["sage_mean"](plan, deg, x.to(device))
    ref = pyg_ref.scatter(x.index_select(0, ei[0]), ei[1], n, reduce="mean")
    torch.testing.assert_close(out.cpu(), ref, rtol=1e-5, atol=1e-5)
