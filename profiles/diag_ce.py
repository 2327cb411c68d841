"""Diagnostic: the fused output mean + CE vs the separate CE on the SAME logits of a SAGE forward."""
import sys

import torch

sys.path.insert(0, "tests")
from test_gpu_fused_ce import _setup  # noqa: E402

from elliptic_gnn_project_amd import _lib  # noqa: E402
from elliptic_gnn_project_amd.train_ops import _ce_operands, _MaskedCE, _ws, _ce_ws_bytes  # noqa: E402

dev = torch.device("cuda:0")
data, model, opt, loss_fn, denom = _setup(dev, dropout=0.0)
model.train()
with loss_fn.target(data.y, data.train_mask, denom):
    logits = model(data.x, data.edge_index)
ce = logits._gnnmp_ce
key, loss_f, buf_f, ws_f = ce
w = loss_fn.full.__closure__  # noqa
lg = logits.detach().clone()
wdev = torch.as_tensor(ce[0][2])  # noqa: F841 (pointer only)
key2, y, m8, ww, inv = _ce_operands(data.y, data.train_mask, next(iter(
    [c.cell_contents for c in loss_fn.full.__closure__ if isinstance(c.cell_contents, dict)]))[dev], denom, dev)
print("keys equal", key == key2, key, key2)
N, C = lg.shape
buf = torch.empty((N, 2 * C), device=dev)
loss = torch.empty((), device=dev)
ws = _ws(_ce_ws_bytes(N), dev)
_lib.call("gnn_masked_ce_f32", N, C, lg.data_ptr(), C, y.data_ptr(), m8.data_ptr(), ww.data_ptr(), float(inv),
          buf.data_ptr() + C * 4, 2 * C, loss.data_ptr(), ws.data_ptr(), ws.numel() * 4, _lib.stream_handle(dev))
torch.cuda.synchronize()
nblk = -(-N // 256)
print("loss fused %.9g separate %.9g" % (float(loss_f), float(loss)))
pf, ps = ws_f[:nblk].cpu(), ws[:nblk].cpu()
d = (pf != ps).nonzero().flatten().tolist()
print("partials differ at", d[:20], "of", nblk)
for b in d[:5]:
    print(b, float(pf[b]), float(ps[b]))
dl_f, dl_s = buf_f[:, C:].cpu(), buf[:, C:].cpu()
rows = (dl_f != dl_s).any(1).nonzero().flatten().tolist()
print("dlogits rows differ", len(rows), rows[:10])
for r in rows[:5]:
    print(r, lg[r].tolist(), dl_f[r].tolist(), dl_s[r].tolist(), int(data.y[r]), bool(data.train_mask[r]))

# per-row: the stashed z of the output layer, one masked row at a time in block 9
import elliptic_gnn_project_amd.train_ops as T  # noqa: E402

stash = {}
orig = T.sage_out_mean_ce


def spy(plan, z, C, bias, target):
    stash.update(plan=plan, z=z.clone(), bias=None if bias is None else bias.clone())
    return orig(plan, z, C, bias, target)


T.sage_out_mean_ce = spy
with loss_fn.target(data.y, data.train_mask, denom):
    logits2 = model(data.x, data.edge_index)
print("relaunch logits equal", torch.equal(logits2, logits))
bad = []
for r in range(9 * 256, 10 * 256):
    if not bool(data.train_mask[r]):
        continue
    m = torch.zeros_like(data.train_mask)
    m[r] = True
    tgt = _ce_operands(data.y, m, ww, 1.0, dev)
    lg1, ce1 = orig(stash["plan"], stash["z"], C, stash["bias"], tgt)
    l_s = torch.empty((), device=dev)
    ws2 = _ws(_ce_ws_bytes(N), dev)
    b2 = torch.empty((N, 2 * C), device=dev)
    _lib.call("gnn_masked_ce_f32", N, C, lg1.data_ptr(), C, tgt[1].data_ptr(), tgt[2].data_ptr(), tgt[3].data_ptr(),
              1.0, b2.data_ptr() + C * 4, 2 * C, l_s.data_ptr(), ws2.data_ptr(), ws2.numel() * 4, _lib.stream_handle(dev))
    if float(ce1[1]) != float(l_s):
        bad.append((r, float(ce1[1]), float(l_s), lg1[r].tolist(), int(data.y[r])))
print("rows with a different loss:", len(bad))
for b in bad[:8]:
    print(b)
