"""Post-processing on the GPU (maskclustering_amd.utils.post_process, mc_pp_run) against the
reference's own post_process outputs (tests/golden/pp_small.npz) and the CPU restatement
(oracle/pp_oracle.py) on seeded synthetic scenes.  Bit-exact: point ids, mask assignment,
coverage (float64), object order."""
import os
from types import SimpleNamespace

import numpy as np
import pytest

from oracle import pp_oracle

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden", "pp_small.npz")


def _pp():
    from maskclustering_amd.utils import post_process
    return post_process


def _node(mask_list, vf, order):
    # point_ids iterates in the recorded list(point_ids) order of the reference process
    return SimpleNamespace(mask_list=list(mask_list), visible_frame=np.asarray(vf, np.float32),
                           point_ids=dict.fromkeys(int(x) for x in order).keys())


def _check(got, want_pts, want_masks):
    gp, gm = got
    assert len(gp) == len(want_pts)
    for k in range(len(want_pts)):
        np.testing.assert_array_equal(np.asarray(gp[k]), np.asarray(want_pts[k], np.int64), err_msg=f"object {k}")
        assert gp[k].dtype == np.int64
        assert gm[k] == want_masks[k], f"object {k} masks"


@pytest.mark.parametrize("case", ["a", "b"])
def test_pp_matches_reference_golden(case):
    z = np.load(GOLD)
    fids = z["frame_ids"].tolist()
    keys = [(fids[c], int(l)) for c, l in zip(z["mpc_col"], z["mpc_label"])]
    mpc = {f"{f}_{m}": set(z["mpc_idx"][z["mpc_off"][i]:z["mpc_off"][i + 1]].tolist()) for i, (f, m) in enumerate(keys)}
    mo, mi = z[case + "_node_mask_off"], z[case + "_node_mask_idx"]
    po, pi_ = z[case + "_node_pt_off"], z[case + "_node_pt_idx"]
    nodes = [_node([keys[q] for q in mi[mo[k]:mo[k + 1]]], z[case + "_node_vf"][k], pi_[po[k]:po[k + 1]])
             for k in range(len(mo) - 1)]
    got = _pp().post_process_objects(nodes, mpc, z["scene"], z["pfm"], fids, float(z[case + "_thr"]))
    oo, oi = z[case + "_obj_pt_off"], z[case + "_obj_pt_idx"]
    qo, qi, qc = z[case + "_obj_mask_off"], z[case + "_obj_mask_idx"], z[case + "_obj_mask_cov"]
    want_pts = [oi[oo[k]:oo[k + 1]] for k in range(len(oo) - 1)]
    want_masks = [[(keys[q][0], keys[q][1], float(c)) for q, c in zip(qi[qo[k]:qo[k + 1]], qc[qo[k]:qo[k + 1]])]
                  for k in range(len(qo) - 1)]
    _check(got, want_pts, want_masks)


def synthetic_pp(seed, P=6000, F=40, n_nodes=30, blob=0.05, nb=60):
    """Blobs of points (some far apart, some touching, isolated noise), nodes over random blob
    subsets in shuffled order, masks over random point subsets in the node's frames, random pfm,
    duplicated nodes (overlap merge) and near-duplicates."""
    rng = np.random.default_rng(seed)
    centers = rng.uniform(0, 4, (nb, 3))
    centers[1::7] = centers[0::7][: len(centers[1::7])] + 0.12        # touching pairs (border ties)
    owner = rng.integers(0, nb, P)
    scene = centers[owner] + rng.normal(0, blob, (P, 3))
    scene[rng.random(P) < 0.02] += rng.uniform(-0.5, 0.5, (1, 3))     # stray points (noise class)
    scene = np.round(scene, 3)                                        # exact-distance ties on a grid
    pfm = rng.random((P, F)) < 0.35
    frame_ids = [int(x) for x in np.arange(F) * 10]
    mpc, nodes = {}, []
    lab = 1
    for k in range(n_nodes):
        bl = rng.choice(nb, size=rng.integers(1, 4), replace=False)
        pts = np.nonzero(np.isin(owner, bl))[0]
        pts = rng.permutation(pts)
        vf = rng.random(F) < 0.4
        vcols = np.nonzero(vf)[0]
        if len(vcols) == 0:
            vf[0] = True
            vcols = np.array([0])
        ml = []
        for _ in range(rng.integers(1, 7)):
            c = int(rng.choice(vcols))
            sel = pts[rng.random(len(pts)) < rng.uniform(0.1, 0.9)]
            extra = rng.integers(0, P, 20)                              # points outside the node
            mpc[f"{frame_ids[c]}_{lab}"] = set(np.concatenate([sel, extra]).tolist())
            ml.append((frame_ids[c], lab))
            lab += 1
        nodes.append((ml, vf, pts))
    nodes += [nodes[i] for i in range(0, n_nodes, 5)]                  # exact duplicates
    return scene, pfm, frame_ids, mpc, nodes


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_pp_matches_oracle_synthetic(seed):
    # seed 3: few blobs shared by many nodes -> many overlapping objects (merge chains, both
    # "i merged away" and "j merged away" decisions in one row)
    scene, pfm, fids, mpc, nodes = synthetic_pp(seed, **(dict(nb=12, n_nodes=50) if seed == 3 else {}))
    thr = [0.5, 0.7, 0.2, 0.3][seed]
    got = _pp().post_process_objects([_node(*n) for n in nodes], mpc, scene, pfm, fids, thr)
    keys = list(mpc.keys())
    kidx = {k: i for i, k in enumerate(keys)}
    col = {f: c for c, f in enumerate(fids)}
    mask_pts = [np.array(sorted(mpc[k]), np.int64) for k in keys]
    mask_col = np.array([col[int(k.rsplit("_", 1)[0])] for k in keys])
    onodes = [([kidx[f"{f}_{m}"] for f, m in ml], vf, pts) for ml, vf, pts in nodes]
    wp, wm = pp_oracle.post_process_objects(scene, pfm, mask_pts, mask_col, onodes, thr)
    want_masks = [[(int(keys[q].rsplit("_", 1)[0]), int(keys[q].rsplit("_", 1)[1]), c) for q, c in ml] for ml in wm]
    assert len(wp) > 3
    _check(got, wp, want_masks)


def test_pp_errors_and_empty():
    pp = _pp()
    scene = np.zeros((10, 3))
    pfm = np.zeros((10, 4), bool)
    assert pp.post_process_objects([], {}, scene, pfm, [0, 1, 2, 3], 0.5) == ([], [])
    one = _node([(0, 1)], [1, 0, 0, 0], [0, 1])                       # < 2 masks: ignored (:182)
    assert pp.post_process_objects([one], {}, scene, pfm, [0, 1, 2, 3], 0.5) == ([], [])
    bad = _node([(0, 1), (1, 2)], [1, 0, 0, 0], [0, 1])               # frame 1 not visible (:69)
    with pytest.raises(IndexError):
        pp.post_process_objects([bad], {"0_1": {0}, "1_2": {1}}, scene, pfm, [0, 1, 2, 3], 0.5)
    missing = _node([(0, 1), (0, 2)], [1, 0, 0, 0], [0, 1])           # no such mask (:70)
    with pytest.raises(KeyError):
        pp.post_process_objects([missing], {"0_1": {0}}, scene, pfm, [0, 1, 2, 3], 0.5)


def test_pp_after_dropin_graph_path():
    """The drop-in graph path's own outputs: the CSR fast path (MaskPointClouds) and a plain dict
    of the same sets give the same objects, equal to the oracle's on the same point orders."""
    import sys
    from conftest import GOLDEN
    sys.path.insert(0, GOLDEN)
    import make_api_golden as ag
    from test_gpu_api import PinholeIntrinsic, _load
    from maskclustering_amd.graph import construction, iterative_clustering
    z, frames, fids, args = _load("api_small_scannet")
    nodes, thr, mpc, pfm = construction.mask_graph_construction(args, frames.scene_points, fids,
                                                                ag.FrameDataset(frames, fids, PinholeIntrinsic))
    objects = iterative_clustering.iterative_clustering(nodes, thr, args.view_consensus_threshold, False)
    assert getattr(mpc, "csr", None) is not None
    fast = _pp().post_process_objects(objects, mpc, frames.scene_points, pfm, fids, 0.5)
    plain = _pp().post_process_objects(objects, dict(mpc), frames.scene_points, pfm, fids, 0.5)
    keys = list(mpc.keys())
    kidx = {k: i for i, k in enumerate(keys)}
    col = {f: c for c, f in enumerate(fids)}
    onodes = [([kidx[f"{f}_{m}"] for f, m in o.mask_list], o.visible_bool(), np.fromiter(o.point_ids, np.int64))
              for o in objects]
    wp, wm = pp_oracle.post_process_objects(np.asarray(frames.scene_points, np.float64), np.asarray(pfm),
                                            [np.fromiter(mpc[k], np.int64) for k in keys],
                                            np.array([col[int(k.rsplit("_", 1)[0])] for k in keys]), onodes, 0.5)
    want_masks = [[(int(keys[q].rsplit("_", 1)[0]), int(keys[q].rsplit("_", 1)[1]), c) for q, c in ml] for ml in wm]
    assert len(wp) > 5
    for got in (fast, plain):
        gm = [[(int(f), int(m), c) for f, m, c in ml] for ml in got[1]]
        _check((got[0], gm), wp, want_masks)
    mpc[keys[0]] = set()                       # any assignment drops the CSR fast path
    assert mpc.csr is None


def _oracle_vs_gpu(scene, pfm, fids, mpc, nodes, thr):
    got = _pp().post_process_objects([_node(*n) for n in nodes], mpc, scene, pfm, fids, thr)
    keys = list(mpc.keys())
    kidx = {k: i for i, k in enumerate(keys)}
    col = {f: c for c, f in enumerate(fids)}
    onodes = [([kidx[f"{f}_{m}"] for f, m in ml], vf, np.asarray(pts, np.int64)) for ml, vf, pts in nodes]
    wp, wm = pp_oracle.post_process_objects(scene, pfm, [np.array(sorted(mpc[k]), np.int64) for k in keys],
                                            np.array([col[k.rsplit("_", 1)[0]] if isinstance(fids[0], str)
                                                      else col[int(k.rsplit("_", 1)[0])] for k in keys]), onodes, thr)
    want = [[(keys[q].rsplit("_", 1)[0] if isinstance(fids[0], str) else int(keys[q].rsplit("_", 1)[0]),
              int(keys[q].rsplit("_", 1)[1]), c) for q, c in ml] for ml in wm]
    _check(got, wp, want)
    return got


def test_pp_edge_cases():
    """Empty node, all-noise node, masks that hold none of the node's points, a single final
    object, string frame ids (TASMap, dataset/tasmap.py:26-34), thresholds 0 and 1."""
    rng = np.random.default_rng(7)
    P, F = 400, 6
    scene = np.round(np.concatenate([rng.normal(0, 0.03, (200, 3)),          # one dense blob
                                     rng.uniform(5, 50, (200, 3))]), 4)     # sparse: all noise
    pfm = rng.random((P, F)) < 0.5
    fids = [f"{i:05d}" for i in range(F)]
    mpc = {f"{fids[0]}_1": set(range(0, 150)), f"{fids[1]}_2": set(range(50, 200)),
           f"{fids[2]}_3": set(range(300, 320)), f"{fids[3]}_4": set(range(390, 400)),
           f"{fids[4]}_5": {0}, f"{fids[5]}_6": set(range(200, 400))}
    vf = np.ones(F, bool)
    nodes = [([(fids[0], 1), (fids[1], 2)], vf, []),                               # empty node
             ([(fids[2], 3), (fids[5], 6)], vf, rng.permutation(np.arange(200, 400))),  # all noise
             ([(fids[3], 4), (fids[4], 5)], vf, rng.permutation(np.arange(0, 200))),  # masks barely touch
             ([(fids[0], 1), (fids[1], 2), (fids[4], 5)], vf, rng.permutation(np.arange(0, 200)))]
    for thr in (0.0, 0.5, 1.0):
        _oracle_vs_gpu(scene, pfm, fids, mpc, nodes, thr)
    got = _oracle_vs_gpu(scene, pfm, fids, mpc, nodes[3:], 0.0)
    assert len(got[0]) == 1 and len(got[1][0]) == 3


@pytest.mark.parametrize("seed", [0, 3])
def test_pp_split_dbscan_path(seed, monkeypatch):
    """Nodes above MC_PP_BIG_MIN points take the split DBSCAN (grid per node, neighbour counts and
    unions on 512-point chunks over the chip, labels per node): same objects as the oracle."""
    monkeypatch.setenv("MC_PP_BIG_MIN", "60")
    scene, pfm, fids, mpc, nodes = synthetic_pp(seed, **(dict(nb=12, n_nodes=50) if seed == 3 else {}))
    _oracle_vs_gpu(scene, pfm, fids, mpc, nodes, 0.5)
    z = np.load(GOLD)
    fids = z["frame_ids"].tolist()
    keys = [(fids[c], int(l)) for c, l in zip(z["mpc_col"], z["mpc_label"])]
    mpc = {f"{f}_{m}": set(z["mpc_idx"][z["mpc_off"][i]:z["mpc_off"][i + 1]].tolist()) for i, (f, m) in enumerate(keys)}
    mo, mi = z["b_node_mask_off"], z["b_node_mask_idx"]
    po, pi_ = z["b_node_pt_off"], z["b_node_pt_idx"]
    nodes = [_node([keys[q] for q in mi[mo[k]:mo[k + 1]]], z["b_node_vf"][k], pi_[po[k]:po[k + 1]])
             for k in range(len(mo) - 1)]
    got = _pp().post_process_objects(nodes, mpc, z["scene"], z["pfm"], fids, float(z["b_thr"]))
    oo, oi = z["b_obj_pt_off"], z["b_obj_pt_idx"]
    assert len(got[0]) == len(oo) - 1
    for k in range(len(oo) - 1):
        np.testing.assert_array_equal(got[0][k], oi[oo[k]:oo[k + 1]].astype(np.int64))


@pytest.mark.parametrize("seed", [1, 3])
def test_pp_device_greedy_merge(seed, monkeypatch):
    """MC_PP_GREEDY_CAP=0 sends every merge decision to the device greedy pass (k_pp_greedy, the
    path for more than 65536 non-zero decisions): same objects as the oracle."""
    monkeypatch.setenv("MC_PP_GREEDY_CAP", "0")
    scene, pfm, fids, mpc, nodes = synthetic_pp(seed, **(dict(nb=12, n_nodes=50) if seed == 3 else {}))
    got = _oracle_vs_gpu(scene, pfm, fids, mpc, nodes, 0.5)
    assert len(got[0]) > 3
