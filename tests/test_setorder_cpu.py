"""mc_setorder_replay (maskclustering_amd/csrc/mc_setorder.inl, host code) against the running
interpreter: the reference's own container building (graph/iterative_clustering.py:5-10 over a
networkx graph made the way from_numpy_array makes it, graph/node.py:24-37's mask_list / set.union /
son_node_info, level-0 sets as set(ndarray) of ascending ids, utils/mask_backprojection.py:147) run
with real CPython sets, on random histories.  Exact: every order must be equal."""
import networkx as nx
import numpy as np
import pytest

from maskclustering_amd import _native


def _reference(levels_edges, level0_sets):
    """levels_edges[t]: (N_t, list of (a, b)); the reference's objects of the last level as
    (mask_list of level-0 indices, list(point_ids), [son member indices]) plus labels per level."""
    nodes = [([i], s, (0, i)) for i, s in enumerate(level0_sets)]
    labels = []
    out = None
    for t, (N, edges) in enumerate(levels_edges):
        assert N == len(nodes)
        G = nx.Graph()
        G.add_nodes_from(range(N))
        both = sorted({(a, b) for a, b in edges} | {(b, a) for a, b in edges})  # A.nonzero(), row-major
        G.add_edges_from(both)
        lab = np.full(N, -1)
        new, sons = [], []
        for comp in nx.connected_components(G):           # iterative_clustering.py:7
            k = len(new)
            mask_list, point_ids, son = [], set(), []
            for i in comp:                                 # graph/node.py:31-36
                ml, pts, info = nodes[i]
                mask_list += ml
                point_ids = point_ids.union(pts)
                son.append(info[1])
                lab[i] = k
            new.append((mask_list, point_ids, (t + 1, k)))
            sons.append(son)
        labels.append(lab)
        nodes = new
        out = [(ml, list(p), s) for (ml, p, _), s in zip(new, sons)]
    return out, labels


def _native_run(levels_edges, level0_seqs, threads=0):
    sizes = [n for n, _ in levels_edges]
    eo = np.zeros(len(levels_edges) + 1, np.int64)
    ea, eb = [], []
    for t, (_, e) in enumerate(levels_edges):
        eo[t + 1] = eo[t] + len(e)
        ea += [a for a, _ in e]
        eb += [b for _, b in e]
    po = np.zeros(len(level0_seqs) + 1, np.int64)
    np.cumsum([len(s) for s in level0_seqs], out=po[1:])
    pts = np.concatenate(level0_seqs) if level0_seqs else np.zeros(0, np.int32)
    return _native.setorder_replay(sizes, eo, ea, eb, po, pts, threads=threads, labels=True)


def _levels(rng, N0, T, p):
    """random graph per iteration; the next level has as many nodes as this one's components"""
    levels = []
    N = N0
    for _ in range(T):
        m = int(rng.poisson(p * N)) if N > 1 else 0
        a = rng.integers(0, N, m)
        b = rng.integers(0, N, m)
        e = sorted({(int(min(x, y)), int(max(x, y))) for x, y in zip(a, b) if x != y})
        rng.shuffle(e)
        levels.append((N, e))
        G = nx.Graph()
        G.add_nodes_from(range(N))
        G.add_edges_from(e)
        N = nx.number_connected_components(G)
    return levels


def _check(levels, seqs, threads=0):
    want, wlab = _reference(levels, [set(np.asarray(s, np.int64)) for s in seqs])
    got = _native_run(levels, seqs, threads)
    assert len(got["mask_off"]) - 1 == len(want)
    for k, (ml, pts, son) in enumerate(want):
        a, b = got["mask_off"][k], got["mask_off"][k + 1]
        assert got["mask_order"][a:b].tolist() == ml, f"object {k}: mask_list order"
        a, b = got["pt_off"][k], got["pt_off"][k + 1]
        assert got["pts"][a:b].tolist() == [int(x) for x in pts], f"object {k}: point_ids order"
        a, b = got["son_off"][k], got["son_off"][k + 1]
        assert got["son_order"][a:b].tolist() == son, f"object {k}: son order"
    np.testing.assert_array_equal(got["labels"], np.concatenate(wlab))


@pytest.mark.parametrize("seed", range(6))
def test_random_histories(seed):
    rng = np.random.default_rng(seed)
    N0 = int(rng.integers(20, 400))
    seqs = []
    for _ in range(N0):
        n = int(rng.choice([0, 1, 3, 4, 5, 20, 77, 300, 1200]))
        base = int(rng.integers(0, 2_000_000))
        kind = rng.integers(0, 3)
        if kind == 0:   # dense range (collision-free home slots)
            ids = base + np.arange(n)
        elif kind == 1:  # spread ids (probing, perturbation)
            ids = rng.choice(4_000_000, n, replace=False)
        else:            # strided: every id on the same residue of a power of two
            ids = base + 1024 * np.arange(n)
        seqs.append(np.unique(ids).astype(np.int32))
    _check(_levels(rng, N0, int(rng.integers(1, 5)), float(rng.choice([0.3, 0.8, 1.5]))), seqs)


def test_large_sets_grow_by_two():
    """unions beyond 50000 entries (set_add_entry's x2 growth) and a component set of > 50000 nodes
    (a chain: BFS discovery in index order)"""
    rng = np.random.default_rng(7)
    seqs = [np.unique(rng.choice(3_000_000, 9000, replace=False)).astype(np.int32) for _ in range(14)]
    _check([(14, [(i, i + 1) for i in range(13)])], seqs)
    N0 = 60000
    seqs = [np.array([i * 7], np.int32) for i in range(N0)]
    edges = [(i, i + 1) for i in range(N0 - 1)]
    rng.shuffle(edges)
    _check([(N0, edges)], seqs)


def test_threads_do_not_change_orders():
    rng = np.random.default_rng(11)
    seqs = [np.unique(rng.choice(500_000, int(rng.integers(0, 900)), replace=False)).astype(np.int32)
            for _ in range(600)]
    levels = _levels(rng, 600, 3, 0.9)
    one, many = _native_run(levels, seqs, 1), _native_run(levels, seqs, 8)
    for k in one:
        np.testing.assert_array_equal(one[k], many[k])


def test_inconsistent_levels_raise():
    with pytest.raises(_native.McError):
        _native.setorder_replay([3, 3], [0, 1, 1], [0], [1], [0, 1, 2, 3], [0, 1, 2])  # 2 components, not 3
    with pytest.raises(_native.McError):
        _native.setorder_replay([3], [0, 1], [0], [0], [0, 1, 2, 3], [0, 1, 2])        # self edge


@pytest.mark.parametrize("cfg", ["scannet", "scannetpp"])
def test_reference_run_orders(cfg):
    """The whole order chain on the CPU against the reference's own main path: the reference's mask
    sets (api_small golden, S1 of the reference's glue) -> the S2-S6 oracle, whose per-iteration edges
    feed mc_setorder_replay -> every final node's list(point_ids) and mask_list equal what the reference's
    own iterative_clustering produced (e2e_pp_small golden, tests/golden/make_e2e_pp_golden.py)."""
    import os
    from conftest import GOLDEN
    from oracle import oracle
    z = np.load(os.path.join(GOLDEN, f"api_small_{cfg}.npz"))
    g = np.load(os.path.join(GOLDEN, f"e2e_pp_small_{cfg}.npz"))
    c = z["cfg"]
    ct = int(c[2]) if bool(z["cfg_ct_is_int"]) else float(c[2])
    P, F = len(z["in_scene"]), len(z["in_frame_ids"])
    col, lab, off, idx = z["mpc_col"], z["mpc_label"], z["mpc_off"], z["mpc_idx"]
    out = oracle.run_sparse(P, F, col, lab, off, idx, mask_visible_threshold=float(c[0]),
                            undersegment_filter_threshold=float(c[1]), view_consensus_threshold=ct,
                            contained_threshold=float(c[3]), edge_cap=1 << 20)
    assert len(out["gl_col"]) == len(col)            # every reference mask is a global mask
    T = int(out["num_iters"])
    tt, aa, bb = out["edges"]
    eo = np.searchsorted(tt, np.arange(T + 1))
    node0 = out["node0_g"]
    po = np.zeros(len(node0) + 1, np.int64)
    np.cumsum(np.diff(off)[node0], out=po[1:])
    seqs = np.concatenate([idx[off[m]:off[m + 1]] for m in node0])
    got = _native.setorder_replay(out["level_sizes"][:T], eo, aa, bb, po, seqs, labels=True)
    np.testing.assert_array_equal(got["labels"], np.concatenate([out[f"part_{t}"] for t in range(T)]))
    fids = z["in_frame_ids"]
    no, ni = g["node_order_off"], g["node_order_idx"]
    assert len(got["pt_off"]) == len(no) > 10
    for k in range(len(no) - 1):
        np.testing.assert_array_equal(got["pts"][got["pt_off"][k]:got["pt_off"][k + 1]], ni[no[k]:no[k + 1]],
                                      err_msg=f"node {k}: list(point_ids)")
        ml = [node0[i] for i in got["mask_order"][got["mask_off"][k]:got["mask_off"][k + 1]]]
        assert ";".join(f"{fids[col[m]]}_{lab[m]}" for m in ml) == str(g["node_mask_lists"][k]), f"node {k} mask_list"


@pytest.mark.parametrize("async_build", [True, False])
def test_begin_finish_on_csr_rows(async_build):
    """mc_setorder_begin / finish (the level-0 sets built on a background thread, read straight from
    rows of a CSR in any order, with rows shared by no node) == mc_setorder_replay on the flattened
    sequences."""
    rng = np.random.default_rng(5)
    rows = [np.unique(rng.choice(800_000, int(rng.integers(0, 700)), replace=False)).astype(np.int32)
            for _ in range(900)]
    off = np.zeros(len(rows) + 1, np.int64)
    np.cumsum([len(r) for r in rows], out=off[1:])
    pts = np.concatenate(rows)
    node_rows = rng.permutation(len(rows))[:700]           # level-0 node i reads CSR row node_rows[i]
    seqs = [rows[r] for r in node_rows]
    levels = _levels(rng, len(seqs), 4, 0.9)
    want = _native_run(levels, seqs)
    so = _native.SetOrder(off[node_rows], off[node_rows + 1] - off[node_rows], pts, async_build=async_build)
    sizes = [n for n, _ in levels]
    eo = np.zeros(len(levels) + 1, np.int64)
    np.cumsum([len(e) for _, e in levels], out=eo[1:])
    ea = np.array([a for _, e in levels for a, _ in e], np.int32)
    eb = np.array([b for _, e in levels for _, b in e], np.int32)
    got = so.finish(sizes, eo, ea, eb, labels=True)
    for k in want:
        np.testing.assert_array_equal(want[k], got[k], err_msg=k)
    with pytest.raises(RuntimeError):
        so.finish(sizes, eo, ea, eb)


def test_begin_rejects_bad_ranges_and_frees_unfinished():
    with pytest.raises(ValueError):
        _native.SetOrder([0], [5], np.arange(3, dtype=np.int32))
    with pytest.raises(_native.McError):  # a negative id: found by the build's workers, reported by finish
        _native.SetOrder([0], [2], np.array([1, -1], np.int32)).finish([1], np.zeros(2, np.int64),
                                                                       np.zeros(0, np.int32), np.zeros(0, np.int32))
    so = _native.SetOrder([0, 2], [2, 1], np.arange(3, dtype=np.int32))
    so.close()  # never finished: the background build is joined and released


def test_replay_in_forked_child():
    """The process-wide worker pool after fork(): a child inherits the pool object but not its threads;
    a replay in the child must build its own pool and finish (it hung in done_.wait before)."""
    import os
    rng = np.random.default_rng(11)
    seqs = [np.unique(rng.choice(5000, int(rng.integers(1, 60)), replace=False)).astype(np.int32) for _ in range(300)]
    levels = _levels(rng, len(seqs), 3, 0.9)
    want = _native_run(levels, seqs, threads=4)  # the parent's pool now exists, with live workers
    r, w = os.pipe()
    pid = os.fork()
    if pid == 0:  # child: same replay, exit status = equal or not
        os.close(r)
        code = 1
        try:
            got = _native_run(levels, seqs, threads=4)
            code = 0 if all(np.array_equal(want[k], got[k]) for k in want) else 2
        finally:
            os.write(w, bytes([code]))
            os._exit(code)
    os.close(w)
    import select
    ready, _, _ = select.select([r], [], [], 60)
    if not ready:
        os.kill(pid, 9)
        os.waitpid(pid, 0)
        pytest.fail("replay in the forked child did not finish within 60 s")
    code = os.read(r, 1)
    os.waitpid(pid, 0)
    assert code == bytes([0]), code
