"""The drop-in modules (maskclustering_amd.graph / .utils, the reference's module
paths and signatures) on the GPU against the REFERENCE's own end-to-end
outputs: graph/construction.py:mask_graph_construction followed by
graph/iterative_clustering.py:iterative_clustering on synthetic RGB-D frames
(tests/golden/make_api_golden.py).  Canonical, order-free comparison."""
import os
import sys
from types import SimpleNamespace

import numpy as np
import pytest

from conftest import GOLDEN

sys.path.insert(0, GOLDEN)
pytestmark = pytest.mark.gpu

CASES = ["api_small_scannet", "api_small_scannetpp"]


class PinholeIntrinsic:
    """The two accessors of open3d.camera.PinholeCameraIntrinsic the path reads."""

    def __init__(self, fx, fy, cx, cy):
        self.f, self.c = (fx, fy), (cx, cy)

    def get_focal_length(self):
        return self.f

    def get_principal_point(self):
        return self.c


def _load(name):
    z = dict(np.load(os.path.join(GOLDEN, name + ".npz")))
    frames = SimpleNamespace(scene_points=z["in_scene"], depth=z["in_depth"], seg=z["in_seg"],
                             intrinsics=z["in_intrinsics"], poses=z["in_poses"])
    fids = z["in_frame_ids"].tolist()
    cfg = z["cfg"]
    ct = int(cfg[2]) if bool(z["cfg_ct_is_int"]) else float(cfg[2])
    args = SimpleNamespace(debug=False, mask_visible_threshold=float(cfg[0]), undersegment_filter_threshold=float(cfg[1]),
                           view_consensus_threshold=ct, contained_threshold=float(cfg[3]))
    return z, frames, fids, args


def _compare(got, want, keys):
    for k in keys:
        np.testing.assert_array_equal(np.asarray(got[k]), want[k], err_msg=k)


ALL = ["mpc_col", "mpc_label", "mpc_off", "mpc_idx", "thr_value", "thr_is_int", "pfm_bits"] + \
      [p + k for p in ("n0_", "obj_") for k in ("mask_off", "mask_idx", "vf_bits", "c_off", "c_idx", "pt_off",
                                               "pt_idx", "node_info", "son_off", "son_idx")]


@pytest.mark.parametrize("name", CASES)
def test_dropin_end_to_end_matches_reference(name):
    import make_api_golden as ag
    from maskclustering_amd.graph import construction, iterative_clustering
    z, frames, fids, args = _load(name)
    ds = ag.FrameDataset(frames, fids, PinholeIntrinsic)
    nodes, thr, mpc, pfm = construction.mask_graph_construction(args, frames.scene_points, fids, ds)
    assert all(isinstance(t, int) and t == 1 or isinstance(t, np.float32) for t in thr)
    objects = iterative_clustering.iterative_clustering(nodes, thr, args.view_consensus_threshold, False)
    got = ag.canonical_outputs(nodes, thr, mpc, pfm, objects, fids)
    _compare(got, z, ALL)


def test_dropin_general_node_path(name="api_small_scannet"):
    """Nodes built by the caller (dense float tensors, like init_nodes does) go through the
    CSR packing path and give the same clusters as the device-graph fast path."""
    import torch
    import make_api_golden as ag
    from maskclustering_amd.graph import construction, iterative_clustering
    from maskclustering_amd.graph.node import Node
    z, frames, fids, args = _load(name)
    ds = ag.FrameDataset(frames, fids, PinholeIntrinsic)
    nodes, thr, mpc, pfm = construction.mask_graph_construction(args, frames.scene_points, fids, ds)
    plain = [Node(n.mask_list, n.visible_frame.clone(), n.contained_mask.clone(), n.point_ids, n.node_info, None)
             for n in nodes]
    assert isinstance(plain[0].visible_frame, torch.Tensor)
    objects = iterative_clustering.iterative_clustering(plain, thr, args.view_consensus_threshold, False)
    got = ag.canonical_outputs(nodes, thr, mpc, pfm, objects, fids)
    _compare(got, z, [k for k in ALL if k.startswith("obj_")])


def test_dropin_frame_backprojection_matches_reference():
    """utils.mask_backprojection.frame_backprojection per frame == the reference's per-frame sets."""
    import make_api_golden as ag
    from maskclustering_amd.utils import mask_backprojection as mb
    z, frames, fids, args = _load("api_small_scannet")
    ds = ag.FrameDataset(frames, fids, PinholeIntrinsic)
    import torch
    scene = torch.tensor(frames.scene_points).float().cuda()  # construction.py:37
    keys = {(int(c), int(l)): k for k, (c, l) in enumerate(zip(z["mpc_col"], z["mpc_label"]))}
    seen = 0
    for c, fid in enumerate(fids):
        info, fpts = mb.frame_backprojection(ds, scene, fid)
        for mid, s in info.items():
            assert isinstance(mid, np.uint8)
            k = keys[(c, int(mid))]
            assert sorted(s) == z["mpc_idx"][z["mpc_off"][k]:z["mpc_off"][k + 1]].tolist()
            seen += 1
        assert set(fpts) == set().union(*info.values()) if info else fpts == []
    assert seen == len(z["mpc_col"])


def _pp_golden(cfg):
    import json
    meta = json.load(open(os.path.join(GOLDEN, "e2e_pp_small.meta.json")))
    # the orders restate networkx 3.x's _plain_bfs set orders (mc_setorder.inl, iterative_clustering._replay)
    assert meta["generated_with"]["networkx"].split(".")[0] == "3", meta
    return np.load(os.path.join(GOLDEN, f"e2e_pp_small_{cfg}.npz"))


def _exports(objects, mpc, frames, pfm, fids, thr):
    from maskclustering_amd.utils import post_process as pp
    pts, masks = pp.post_process_objects(objects, mpc, frames.scene_points, np.asarray(pfm), fids, thr)
    return [np.asarray(p, np.int64) for p in pts], [[(str(f), int(m), float(c)) for f, m, c in ml] for ml in masks]


def _golden_exports(g):
    oo, oi = g["obj_pt_off"], g["obj_pt_idx"]
    qo = g["obj_mask_off"]
    pts = [oi[oo[k]:oo[k + 1]].astype(np.int64) for k in range(len(oo) - 1)]
    masks = [[(str(f), int(m), float(c)) for f, m, c in zip(g["obj_mask_frame"][qo[k]:qo[k + 1]],
                                                          g["obj_mask_id"][qo[k]:qo[k + 1]],
                                                          g["obj_mask_cov"][qo[k]:qo[k + 1]])]
             for k in range(len(qo) - 1)]
    return pts, masks


def _check_reference_orders(objects, g):
    no, ni = g["node_order_off"], g["node_order_idx"]
    assert len(objects) == len(no) - 1
    for k, o in enumerate(objects):
        assert [int(x) for x in o.point_ids] == ni[no[k]:no[k + 1]].tolist(), f"node {k} point order"
        assert ";".join(f"{f}_{m}" for f, m in o.mask_list) == str(g["node_mask_lists"][k]), f"node {k} mask_list"


@pytest.mark.parametrize("cfg", ["scannet", "scannetpp"])
def test_dropin_main_path_exports_match_reference(cfg):
    """main.py:17-21 through the drop-ins in their DEFAULT mode (S1 -> S6 -> post_process) exports
    exactly what the reference's own run exports (tests/golden/make_e2e_pp_golden.py): the same
    objects in the same order, their point ids in the same order, the same mask lists and
    coverages; every final node's list(point_ids) is the reference's iteration order (the native
    set-order restatement, mc_setorder_replay)."""
    import make_api_golden as ag
    from maskclustering_amd.graph import construction, iterative_clustering
    z, frames, fids, args = _load(f"api_small_{cfg}")
    g = _pp_golden(cfg)
    nodes, thr, mpc, pfm = construction.mask_graph_construction(args, frames.scene_points, fids,
                                                                ag.FrameDataset(frames, fids, PinholeIntrinsic))
    objects = iterative_clustering.iterative_clustering(nodes, thr, args.view_consensus_threshold, False)
    _check_reference_orders(objects, g)
    gp, gm = _exports(objects, mpc, frames, pfm, fids, float(g["pp_thr"]))
    wp, wm = _golden_exports(g)
    assert len(gp) == len(wp) > 5
    for k in range(len(wp)):
        np.testing.assert_array_equal(gp[k], wp[k], err_msg=f"object {k}")
        assert gm[k] == wm[k], f"object {k} masks"


@pytest.mark.parametrize("cfg", ["scannet", "scannetpp"])
def test_dropin_general_nodes_reference_orders(cfg):
    """Node objects built by the caller (point sets of unknown history) take the Python-set replay
    of the same steps: the same reference orders."""
    import make_api_golden as ag
    from maskclustering_amd.graph import construction, iterative_clustering
    from maskclustering_amd.graph.node import Node
    z, frames, fids, args = _load(f"api_small_{cfg}")
    g = _pp_golden(cfg)
    nodes, thr, mpc, pfm = construction.mask_graph_construction(args, frames.scene_points, fids,
                                                                ag.FrameDataset(frames, fids, PinholeIntrinsic))
    plain = [Node(n.mask_list, n.visible_frame.clone(), n.contained_mask.clone(), n.point_ids, n.node_info, None)
             for n in nodes]
    objects = iterative_clustering.iterative_clustering(plain, thr, args.view_consensus_threshold, False)
    _check_reference_orders(objects, g)


@pytest.mark.parametrize("cfg", ["scannet", "scannetpp"])
def test_dropin_canonical_exports(cfg):
    """replay=False (canonical: no edge capture, no host replay): the containers hold the reference's
    contents in another order; on these scenes the exported objects still equal the reference's as
    sets of point sets with the same mask lists (order-free comparison)."""
    import make_api_golden as ag
    from maskclustering_amd.graph import construction, iterative_clustering
    z, frames, fids, args = _load(f"api_small_{cfg}")
    g = _pp_golden(cfg)
    nodes, thr, mpc, pfm = construction.mask_graph_construction(args, frames.scene_points, fids,
                                                                ag.FrameDataset(frames, fids, PinholeIntrinsic))
    objects = iterative_clustering.iterative_clustering(nodes, thr, args.view_consensus_threshold, False,
                                                        replay=False)
    gp, gm = _exports(objects, mpc, frames, pfm, fids, float(g["pp_thr"]))
    wp, wm = _golden_exports(g)
    got = sorted((tuple(sorted(p.tolist())), tuple(sorted(m))) for p, m in zip(gp, gm))
    want = sorted((tuple(sorted(p.tolist())), tuple(sorted(m))) for p, m in zip(wp, wm))
    assert got == want
