"""CPU: the K11 sampling oracle (oracle/neighbor_sample.py) against PyG NeighborLoader semantics.

PyG's draws are not reproducible (pyg-lib RNG), so the oracle is pinned where PyG is
deterministic: with num_neighbors = -1 on every hop the batch is the k-hop in-neighbourhood,
stated independently as a BFS (khop_known_answer) — node order, edge set, hop counts.  For
finite fan-outs the checks are the sampling contract (bounds, no replacement, uniformity).
"""
import numpy as np
import pytest

from oracle import neighbor_sample as NS


def _graph(n, e, seed, hub=None):
    rng = np.random.default_rng(seed)
    src = rng.integers(0, n, e)
    dst = rng.integers(0, n, e)
    if hub is not None:  # a hub with many in-edges (duplicates and a self loop included)
        k = 60
        src = np.concatenate([src, rng.integers(0, n, k), [hub]])
        dst = np.concatenate([dst, np.full(k, hub), [hub]])
    return np.stack([src, dst])


@pytest.mark.parametrize("hops", [1, 2, 3])
def test_full_fanout_equals_khop_bfs(hops):
    ei = _graph(60, 150, 1, hub=7)
    seeds = [7, 3, 41, 0]
    n_id, eil, e_id, hn, he = NS.neighbor_sample(ei, 60, seeds, [-1] * hops, seed=5)
    order, edges = NS.khop_known_answer(ei, 60, seeds, hops)
    assert n_id.tolist() == order
    got = sorted(zip(n_id[eil[0]].tolist(), n_id[eil[1]].tolist(), e_id.tolist()))
    assert got == sorted(edges)
    assert sum(hn) == len(order) and sum(he) == len(edges)
    # edges point neighbour -> frontier node, e_id names the original edge
    assert np.array_equal(ei[0][e_id], n_id[eil[0]]) and np.array_equal(ei[1][e_id], n_id[eil[1]])


def test_fanout_bounds_and_no_replacement():
    ei = _graph(80, 400, 2, hub=11)
    n_id, eil, e_id, hn, he = NS.neighbor_sample(ei, 80, [11, 5, 9], [4, 3], seed=123)
    indeg = np.bincount(ei[1], minlength=80)
    start = 0
    for h, k in enumerate([4, 3]):
        seg = slice(start, start + he[h])
        dsts, eids = eil[1][seg], e_id[seg]
        for d in np.unique(dsts):
            picked = eids[dsts == d]
            assert len(picked) == min(k, indeg[n_id[d]])
            assert len(set(picked.tolist())) == len(picked)  # no replacement
        start += he[h]
    assert len(set(n_id.tolist())) == len(n_id)


def test_uniform_selection():
    """Floyd over the hash: every CSR position of a degree-12 row is drawn with p = k/deg."""
    counts = np.zeros(12)
    trials = 3000
    for s in range(trials):
        for p in NS.pick_positions(12, 3, seed=s, hop=0, node=4):
            counts[p] += 1
    freq = counts / trials
    assert np.all(np.abs(freq - 3 / 12) < 0.035), freq


def test_uniform_selection_above_floyd_buffer():
    """More than 256 picks (selection sampling): exactly k distinct positions, ascending, each
    position of a degree-400 row drawn with p = k/deg."""
    deg, k, trials = 400, 300, 400
    counts = np.zeros(deg)
    for s in range(trials):
        picks = NS.pick_positions(deg, k, seed=s, hop=1, node=9)
        assert len(picks) == k and picks == sorted(set(picks)) and 0 <= picks[0] and picks[-1] < deg
        counts[picks] += 1
    freq = counts / trials
    assert abs(freq.mean() - k / deg) < 1e-12
    assert np.all(np.abs(freq - k / deg) < 0.1), freq


def test_duplicate_seeds_rejected():
    with pytest.raises(ValueError):
        NS.neighbor_sample(_graph(10, 20, 3), 10, [1, 1], [2], seed=0)
