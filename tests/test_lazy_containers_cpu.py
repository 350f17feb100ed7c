"""The drop-in construction's lazy containers behave like the reference's plain ones
(graph/construction.py:57 mask_point_clouds dict of sets, :66-78 level-0 node point_ids aliasing
those sets, :40,52 the bool point_frame_matrix)."""
import numpy as np
import pytest

from maskclustering_amd.graph.construction import MaskPointClouds, PointFrameMatrix
from maskclustering_amd.graph.node import Level0Source, Node, level0_masks
from maskclustering_amd.pipeline import bool_to_bits


def _plain_and_lazy(seed=0, n=40):
    rng = np.random.default_rng(seed)
    keys = [f"{10 * (i // 3)}_{i % 3 + 1}" for i in range(n)]
    rows = [np.unique(rng.integers(0, 500, rng.integers(0, 30))).astype(np.int32) for _ in keys]
    off = np.zeros(n + 1, np.int64)
    np.cumsum([len(r) for r in rows], out=off[1:])
    pts = np.concatenate(rows)
    plain = {k: set(r.tolist()) for k, r in zip(keys, rows)}
    return keys, plain, MaskPointClouds.from_csr(keys, off, pts)


def test_reads_match_plain_dict():
    keys, plain, lazy = _plain_and_lazy()
    assert len(lazy) == len(plain)
    assert keys[5] in lazy and "nope" not in lazy
    assert lazy[keys[7]] == plain[keys[7]]          # one set made out of order
    assert lazy.get(keys[3]) == plain[keys[3]] and lazy.get("nope", 1) == 1
    assert list(lazy) == list(plain)                # insertion order kept
    assert list(lazy.items()) == list(plain.items())
    assert lazy == plain
    with pytest.raises(KeyError):
        lazy["nope"]


def test_repeated_frame_id_keeps_first_position_and_last_set():
    """a frame id listed twice (construction.py:57 assigns the key twice: first position, last set)"""
    import pickle
    rng = np.random.default_rng(4)
    keys = ["0_1", "0_2", "10_1", "0_1", "20_3", "10_1"]
    rows = [np.unique(rng.integers(0, 100, 12)).astype(np.int32) for _ in keys]
    off = np.zeros(len(keys) + 1, np.int64)
    np.cumsum([len(r) for r in rows], out=off[1:])
    plain = {}
    for k, r in zip(keys, rows):
        plain[k] = set(r.tolist())
    lazy = MaskPointClouds.from_csr(keys, off, np.concatenate(rows))
    assert len(lazy) == len(plain) == 4
    assert lazy["0_1"] == plain["0_1"]
    assert list(lazy) == list(plain) and list(lazy.items()) == list(plain.items())
    assert pickle.loads(pickle.dumps(lazy)) == plain
    lazy2 = MaskPointClouds.from_csr(keys, off, np.concatenate(rows))
    np.save("/dev/null", np.array([lazy2], dtype=object), allow_pickle=True)
    lazy2["new"] = {1}
    plain2 = dict(plain)
    plain2["new"] = {1}
    assert list(lazy2) == list(plain2) and lazy2 == plain2
    del lazy2["10_1"]
    del plain2["10_1"]
    assert list(lazy2.values()) == list(plain2.values())


def test_mutation_drops_csr_and_keeps_order():
    keys, plain, lazy = _plain_and_lazy(1)
    assert lazy.csr is not None
    lazy["new"] = {1, 2}
    plain["new"] = {1, 2}
    assert lazy.csr is None
    assert list(lazy) == list(plain) and lazy == plain
    del lazy[keys[0]]
    del plain[keys[0]]
    assert list(lazy.keys()) == list(plain.keys())


def test_level0_point_ids_alias_the_first_set():
    keys, plain, lazy = _plain_and_lazy(2)
    gl = [(int(k.split("_")[0]), np.uint8(k.split("_")[1])) for k in keys]
    vf = np.arange(len(keys) * 3).reshape(-1, 3) % 2 == 0
    c_off = np.arange(len(keys) + 1, dtype=np.int64)
    c_idx = np.arange(len(keys), dtype=np.int32)[::-1].copy()
    src = Level0Source(gl, keys, vf, c_off, c_idx, 40, lazy)
    node = Node.level0(src, 0, 4, None)
    other = Node.level0(src, 1, 6, None)
    assert node.point_ids is lazy[keys[4]]           # the same object, as init_nodes stores it
    lazy[keys[6]] = {999}                            # replaced before the node's first read
    assert other.point_ids == plain[keys[6]]
    node.point_ids = {1}
    assert node.point_ids == {1}
    assert level0_masks(other) == (gl[6],) and "mask_list" not in other.__dict__
    assert other.mask_list == [gl[6]] and other.node_info == (0, 1) and other.son_node_info is None
    np.testing.assert_array_equal(other.visible_bool(), vf[6])
    np.testing.assert_array_equal(other.contained_ids(), c_idx[6:7])
    assert other.num_masks() == 40
    other.mask_list.append("x")                      # the attribute is a real list once read
    assert level0_masks(other) == [gl[6], "x"]
    with pytest.raises(AttributeError):
        other.no_such_attribute


def test_point_frame_matrix_carries_bits():
    rng = np.random.default_rng(3)
    b = rng.random((50, 70)) < 0.3
    words = bool_to_bits(b)
    pfm = PointFrameMatrix.from_bits(words, 70)
    np.testing.assert_array_equal(np.asarray(pfm), b)
    assert pfm.dtype == bool and not pfm.flags.writeable
    np.testing.assert_array_equal(pfm._mc_bits, words)
    assert pfm[:10]._mc_bits is None and (pfm | pfm)._mc_bits is None


def test_merged_node_points_made_on_first_read():
    arr = np.array([5, 9, 11], np.int32)
    n = Node.compact_lazy_points([(0, 1), (10, 2)], np.ones(4, bool), np.array([0, 1], np.int32), 8, arr, (3, 0),
                                 {(2, 0)})
    assert "_point_ids" not in n.__dict__
    assert n.point_ids == {5, 9, 11} and n.point_ids is n.point_ids
    assert n.mask_list == [(0, 1), (10, 2)] and n.node_info == (3, 0) and n.son_node_info == {(2, 0)}


def test_level0_sequences_detects_same_length_edits():
    """A materialised level-0 set changed in place to the same length (one id removed, another added)
    must send iterative_clustering to the Python replay (the native one would rebuild the set from the
    CSR row and ignore the edit); untouched and read-only sets keep the native path."""
    import types
    from maskclustering_amd.graph.iterative_clustering import _level0_sequences
    pts = np.array([1, 4, 9, 2, 3, 7, 8], np.int32)
    off = np.array([0, 3, 7], np.int64)
    row_of = {"a": 0, "b": 1}
    mpc = types.SimpleNamespace(csr=(row_of, off, pts), _made={})
    h = types.SimpleNamespace(src=types.SimpleNamespace(mpc=mpc, keys=["a", "b"]), node0=np.array([0, 1]))
    st, ln, pp = _level0_sequences(h)
    np.testing.assert_array_equal(st, [0, 3])
    np.testing.assert_array_equal(ln, [3, 4])
    mpc._made["b"] = {2, 3, 7, 8}                 # read, unchanged
    assert _level0_sequences(h) is not None
    mpc._made["b"] = {2, 3, 7, 100}               # same length, one id replaced
    assert _level0_sequences(h) is None
    mpc._made["b"] = {2, 3, 7}                    # shorter
    assert _level0_sequences(h) is None


def test_fast_path_needs_the_untouched_level0_list():
    """iterative_clustering takes the device-graph path only for the very level-0 Node objects the
    construction returned, in order, none with a replaced visible_frame / contained_mask."""
    from maskclustering_amd.graph import construction
    from maskclustering_amd.graph.iterative_clustering import _fast_path
    saved = construction._current["token"]
    try:
        h = construction.GraphHandle(12345, 3, 4, 5, 6)
        nodes = [Node.level0(None, i, i, h) for i in range(3)]
        h.nodes = tuple(nodes)
        construction._current["token"] = 12345
        assert _fast_path(nodes) is h and _fast_path(list(nodes)) is h
        assert _fast_path(nodes[::-1]) is None and _fast_path(nodes[:2]) is None
        assert _fast_path([nodes[0], nodes[1], Node.level0(None, 2, 2, h)]) is None
        construction._current["token"] = 7            # another graph was built since
        assert _fast_path(nodes) is None
        construction._current["token"] = 12345
        nodes[1].contained_mask = None                # a caller-replaced containment row
        assert _fast_path(nodes) is None
    finally:
        construction._current["token"] = saved
