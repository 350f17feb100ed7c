"""Golden fixtures for the post-processing row: the REFERENCE's
own ``utils/post_process.py`` (``post_process`` :173-195 -> ``dbscan_process`` :104-123,
``filter_point`` :40-101, ``merge_overlapping_objects`` :7-37) run on the nodes that the
reference's own graph path produces for synthetic RGB-D frames.

Run ONLY in the build container, where /root/reference exists:

    python tests/golden/make_pp_golden.py

Open3D's ``cluster_dbscan`` / ``select_by_index`` / the PointCloud container are served by
the restatements in make_s1_golden.py (Open3D's DBSCAN loop taken literally; parity of the
library arithmetic unpinned).  ``export`` (:148-170, file output only) is
replaced by a function that captures its two lists.  Everything else is the reference's
unmodified code.  The result depends on the iteration order of each node's point set
(``list(self.point_ids)``, graph/node.py:45), so the fixture records that order as the
reference process saw it, and the tests hand the same order to the drop-in.

Two cases: ``a`` = the final clustered objects (scannet config, point_filter_threshold 0.5);
``b`` = a stress list built from the same objects with the reference's own
``Node.create_node_from_list``: pairs of objects merged into one node (DBSCAN must split
them), duplicates of objects (merge_overlapping_objects must drop them), threshold 0.7.
Outputs are data (inputs and the reference's outputs); no source is copied.
"""
from __future__ import annotations

import os
import sys
from types import SimpleNamespace

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)

import make_api_golden as apig  # noqa: E402
import make_s1_golden as s1g  # noqa: E402


def run_reference_graph(fr, frame_ids):
    mb, torch = s1g._import_reference()
    os.environ["TQDM_DISABLE"] = "1"
    from graph import construction, iterative_clustering  # noqa: E402
    ds = apig.FrameDataset(fr, frame_ids, s1g._Intrinsic)
    args = SimpleNamespace(debug=False, **apig.CONFIGS["scannet"])
    nodes, thr, mpc, pfm = construction.mask_graph_construction(args, fr.scene_points, list(frame_ids), ds)
    objects = iterative_clustering.iterative_clustering(list(nodes), thr, args.view_consensus_threshold, False)
    return objects, mpc, pfm


def run_reference_post_process(node_list, mpc, scene_points, pfm, frame_ids, thr):
    from utils import post_process as pp  # noqa: E402
    got = {}

    def capture(dataset, total_point_ids_list, total_mask_list, args):
        got["pts"] = [np.asarray(p) for p in total_point_ids_list]
        got["masks"] = [list(m) for m in total_mask_list]

    pp.export = capture
    args = SimpleNamespace(debug=False, point_filter_threshold=thr)
    orders = [list(n.point_ids) for n in node_list]   # the order get_point_cloud sees (graph/node.py:45)
    pp.post_process(None, node_list, mpc, scene_points, pfm, list(frame_ids), args)
    return orders, got


def stress_nodes(objects):
    from graph.node import Node  # the reference's own (stubbed open3d import only)
    objs = [o for o in objects if len(o.mask_list) >= 1]
    cen = np.array([np.mean(np.asarray(sorted(o.point_ids)), dtype=np.float64) for o in objs])
    out = list(objs[: len(objs) // 2])
    k = 0
    for i in range(0, len(objs) - 1, 3):                       # merged pairs (two blobs per node)
        out.append(Node.create_node_from_list([objs[i], objs[i + 1]], (99, k)))
        k += 1
    for i in range(0, len(objs), 4):                           # duplicates (overlap ratio 1.0)
        out.append(Node.create_node_from_list([objs[i]], (98, k)))
        k += 1
    del cen
    return out


def pack_case(prefix, node_list, orders, got, key, frame_col):
    out = {}
    mo, mi, vfb, po, pi_ = [0], [], [], [0], []
    for n, order in zip(node_list, orders):
        mi.extend(key(f, m) for f, m in n.mask_list)
        mo.append(len(mi))
        vfb.append(np.asarray(n.visible_frame.cpu() if hasattr(n.visible_frame, "cpu") else n.visible_frame) > 0)
        pi_.extend(int(x) for x in order)
        po.append(len(pi_))
    out[prefix + "node_mask_off"], out[prefix + "node_mask_idx"] = np.array(mo, np.int64), np.array(mi, np.int32)
    out[prefix + "node_vf"] = np.array(vfb, bool)
    out[prefix + "node_pt_off"], out[prefix + "node_pt_idx"] = np.array(po, np.int64), np.array(pi_, np.int32)
    oo, oi, qo, qi, qc = [0], [], [0], [], []
    for pts, ml in zip(got["pts"], got["masks"]):
        oi.extend(int(x) for x in pts)
        oo.append(len(oi))
        for f, m, cov in ml:
            qi.append(key(f, m))
            qc.append(float(cov))
        qo.append(len(qi))
    out[prefix + "obj_pt_off"], out[prefix + "obj_pt_idx"] = np.array(oo, np.int64), np.array(oi, np.int32)
    out[prefix + "obj_mask_off"], out[prefix + "obj_mask_idx"] = np.array(qo, np.int64), np.array(qi, np.int32)
    out[prefix + "obj_mask_cov"] = np.array(qc, np.float64)
    return out


def main():
    from maskclustering_amd.synthetic_frames import make_frames_shape
    fr = make_frames_shape("small", seed=4)
    frame_ids = [int(x) for x in np.arange(0, 10 * fr.num_frames, 10)]
    objects, mpc, pfm = run_reference_graph(fr, frame_ids)
    col = {fid: c for c, fid in enumerate(frame_ids)}
    keys = sorted(mpc.keys(), key=lambda k: (col[int(k.rsplit("_", 1)[0])], int(k.rsplit("_", 1)[1])))
    kidx = {k: i for i, k in enumerate(keys)}

    def key(f, m):
        return kidx[f"{f}_{m}"]

    out = dict(scene=np.asarray(fr.scene_points, np.float64), frame_ids=np.array(frame_ids),
               pfm=np.asarray(pfm, bool))
    out["mpc_col"] = np.array([col[int(k.rsplit("_", 1)[0])] for k in keys], np.int32)
    out["mpc_label"] = np.array([int(k.rsplit("_", 1)[1]) for k in keys], np.int32)
    mo, mi = [0], []
    for k in keys:
        mi.extend(sorted(int(x) for x in mpc[k]))
        mo.append(len(mi))
    out["mpc_off"], out["mpc_idx"] = np.array(mo, np.int64), np.array(mi, np.int32)
    cases = {"a": (list(objects), 0.5), "b": (stress_nodes(objects), 0.7)}
    for name, (nl, thr) in cases.items():
        orders, got = run_reference_post_process(nl, mpc, fr.scene_points, pfm, frame_ids, thr)
        out.update(pack_case(name + "_", nl, orders, got, key, col))
        out[name + "_thr"] = np.array(thr)
        print(f"case {name}: nodes={len(nl)} (>=2 masks: {sum(len(n.mask_list) >= 2 for n in nl)}) "
              f"objects out={len(got['pts'])} points out={sum(len(p) for p in got['pts'])}")
    path = os.path.join(HERE, "pp_small.npz")
    np.savez_compressed(path, **out)
    print(f"-> {path} {os.path.getsize(path) / 1e6:.2f} MB")


if __name__ == "__main__":
    main()
