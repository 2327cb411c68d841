"""CPU restatement of K11 neighbour sampling (TEST INFRASTRUCTURE — never imported by the product).

Follows the reference's mini-batch path: ``NeighborLoader(data, num_neighbors=fanout,
batch_size, input_nodes, shuffle)`` at src/train_gnn.py:329-348 (torch_geometric 2.5.3 with
pyg-lib ``neighbor_sample``: CSC over in-edges, ``replace=False``, ``disjoint=False``,
``subgraph_type='directional'``), consumed by ``train_epoch_minibatch`` (:212-245).

What is PyG's contract and what is ours:
* PyG: hop h samples up to fanout[h] in-neighbours (sources j of edges j -> i) of every node
  first discovered in hop h-1 (the seeds for hop 0), without replacement, all of them when the
  in-degree is <= fanout; nodes are de-duplicated across the batch, seeds first, then new nodes
  in order of appearance; the subgraph's edges point neighbour -> frontier node.  With
  fanout = -1 everywhere the result is the deterministic k-hop in-neighbourhood, which
  ``khop_known_answer`` states independently (a BFS) — the PyG-semantics known answer.
* Ours: WHICH fanout-subset is drawn comes from a counter hash of (seed, hop, node, draw) and
  Floyd's algorithm (csrc/sample.hip; selection sampling, Knuth's algorithm S, above 256 picks),
  picks emitted in ascending CSR position; this module
  reproduces those draws bit for bit so the HIP sampler is checked exactly.  PyG's RNG stream
  (pyg-lib) is not reproducible: the choice of subset is "parity unpinned" against PyG.
Pure Python loops: small graphs only.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np

M64 = (1 << 64) - 1


def sample_hash(seed: int, hop: int, node: int, draw: int) -> int:
    """csrc/sample.hip sample_hash: splitmix64 finaliser over a (seed, hop, node, draw) counter."""
    z = (seed ^ ((0x9E3779B97F4A7C15 * ((hop << 32) | node)) & M64) ^ ((draw * 0xD1B54A32D192ED03) & M64)) & M64
    z ^= z >> 30
    z = (z * 0xBF58476D1CE4E5B9) & M64
    z ^= z >> 27
    z = (z * 0x94D049BB133111EB) & M64
    z ^= z >> 31
    return z >> 32


def csr_by_target(edge_index: np.ndarray, num_nodes: int) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Stable CSR by target (PyG edge order inside a row): rowptr, col (sources), eid."""
    src, dst = np.asarray(edge_index[0], np.int64), np.asarray(edge_index[1], np.int64)
    order = np.argsort(dst, kind="stable")
    rowptr = np.zeros(num_nodes + 1, np.int64)
    np.add.at(rowptr, dst + 1, 1)
    return np.cumsum(rowptr), src[order], order


def pick_positions(deg: int, k: int, seed: int, hop: int, node: int) -> List[int]:
    """CSR positions sampled from a row of ``deg`` slots (k < 0: all)."""
    c = deg if k < 0 else min(deg, k)
    if c == deg:
        return list(range(deg))
    if c > 256:  # more picks than the kernel's Floyd buffer: selection sampling (algorithm S)
        out, need = [], c
        for j in range(deg):
            if need == 0:
                break
            if (sample_hash(seed, hop, node, j) * (deg - j)) >> 32 < need:
                out.append(j)
                need -= 1
        return out
    sel: List[int] = []
    for j in range(deg - c, deg):
        t = (sample_hash(seed, hop, node, j) * (j + 1)) >> 32
        sel.append(j if t in sel else t)
    return sorted(sel)


def neighbor_sample(edge_index: np.ndarray, num_nodes: int, seeds: Sequence[int], fanout: Sequence[int],
                    seed: int):
    """-> n_id, (e_src, e_dst) local, e_id, hop_nodes, hop_edges (the K11 outputs)."""
    rowptr, col, eid = csr_by_target(edge_index, num_nodes)
    n_id = [int(s) for s in seeds]
    if len(set(n_id)) != len(n_id):
        raise ValueError("seed nodes must be distinct")
    local = {v: i for i, v in enumerate(n_id)}
    e_src, e_dst, e_id = [], [], []
    hop_nodes, hop_edges = [len(n_id)], []
    fbeg, fend = 0, len(n_id)
    for h, k in enumerate(fanout):
        hop_src = []
        for i in range(fbeg, fend):
            v = n_id[i]
            r0, d = int(rowptr[v]), int(rowptr[v + 1] - rowptr[v])
            for pos in pick_positions(d, int(k), seed, h, v):
                hop_src.append(int(col[r0 + pos]))
                e_dst.append(i)
                e_id.append(int(eid[r0 + pos]))
        new = 0
        for u in hop_src:  # first appearance order
            if u not in local:
                local[u] = len(n_id)
                n_id.append(u)
                new += 1
        e_src.extend(local[u] for u in hop_src)
        hop_edges.append(len(hop_src))
        hop_nodes.append(new)
        fbeg, fend = fend, len(n_id)
    return (np.array(n_id, np.int64), np.array([e_src, e_dst], np.int64).reshape(2, -1),
            np.array(e_id, np.int64), hop_nodes, hop_edges)


def khop_known_answer(edge_index: np.ndarray, num_nodes: int, seeds: Sequence[int], hops: int):
    """PyG NeighborLoader with num_neighbors = [-1] * hops, stated as a BFS over in-edges:
    the node ORDER (seeds, then each hop's new nodes by first appearance over the frontier's
    in-edges in edge order) and the EDGE SET (every in-edge of every expanded node)."""
    src, dst = np.asarray(edge_index[0]), np.asarray(edge_index[1])
    order = [int(s) for s in seeds]
    seen = set(order)
    frontier = list(order)
    edges = []
    for _ in range(hops):
        nxt = []
        for v in frontier:
            for e in np.nonzero(dst == v)[0]:  # in-edges of v, in edge order
                u = int(src[e])
                edges.append((u, v, int(e)))
                if u not in seen:
                    seen.add(u)
                    order.append(u)
                    nxt.append(u)
        frontier = nxt
    return order, edges
