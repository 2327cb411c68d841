"""ORACLE (test infrastructure only) — pure-Python loop forms for tiny graphs.

An independent second restatement of PyG 2.5.3's aggregation semantics, written edge by
edge in float64 with no tensor ops, used to cross-check oracle/pyg_ref.py on small
inputs (tests/test_oracle_kat.py).  Semantics restated (see pyg_ref.py's header):
  mean:  out_i = (sum over edges e with dst(e)=i of x[src(e)]) / max(#such edges, 1)
  gcn:   remove every loop, append one loop per node; deg_i = #edges into i;
         out_i = sum_e deg_src^-1/2 * deg_i^-1/2 * h[src(e)]
  gat:   remove loops, append loops; e = leaky_relu(a_s[src] + a_d[i]);
         alpha = exp(e - max) / (sum exp + 1e-16) per (i, head); out_i = sum alpha * h[src]
"""
from __future__ import annotations

import math


def mean_agg(x, edges, n):
    f = len(x[0]) if x else 0
    out = [[0.0] * f for _ in range(n)]
    cnt = [0] * n
    for s, d in edges:
        cnt[d] += 1
        for c in range(f):
            out[d][c] += x[s][c]
    return [[v / max(cnt[i], 1) for v in out[i]] for i in range(n)]


def loops_replaced(edges, n):
    return [(s, d) for s, d in edges if s != d] + [(i, i) for i in range(n)]


def gcn_agg(h, edges, n):
    ed = loops_replaced(edges, n)
    deg = [0] * n
    for _, d in ed:
        deg[d] += 1
    dinv = [1.0 / math.sqrt(v) if v > 0 else 0.0 for v in deg]
    f = len(h[0])
    out = [[0.0] * f for _ in range(n)]
    for s, d in ed:
        w = dinv[s] * dinv[d]
        for c in range(f):
            out[d][c] += w * h[s][c]
    return out


def gat_agg(xh, a_s, a_d, edges, n, heads, chans, concat=True, slope=0.2):
    """xh: [n][heads*chans]; a_s, a_d: [n][heads]."""
    ed = loops_replaced(edges, n)
    out = [[0.0] * (heads * chans) for _ in range(n)]
    alphas = {}
    for h in range(heads):
        e = [(s, d, (lambda z: z if z > 0 else z * slope)(a_s[s][h] + a_d[d][h])) for s, d in ed]
        mx = [-math.inf] * n
        for _, d, v in e:
            mx[d] = max(mx[d], v)
        sm = [0.0] * n
        for _, d, v in e:
            sm[d] += math.exp(v - mx[d])
        for k, (s, d, v) in enumerate(e):
            a = math.exp(v - mx[d]) / (sm[d] + 1e-16)
            alphas[(k, h)] = a
            for c in range(chans):
                out[d][h * chans + c] += a * xh[s][h * chans + c]
    if not concat:
        out = [[sum(row[h * chans + c] for h in range(heads)) / heads for c in range(chans)] for row in out]
    return out, alphas
