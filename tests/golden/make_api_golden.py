"""Golden fixtures for the drop-in API: the REFERENCE's own
``mask_graph_construction`` + ``iterative_clustering`` (graph/construction.py:7-20,
graph/iterative_clustering.py:36-43) run end to end on synthetic RGB-D frames.

Run ONLY in the build container, where /root/reference exists:

    python tests/golden/make_api_golden.py

The S1 library calls (Open3D, pytorch3d) are served by the restatements of
make_s1_golden.py; everything else is the reference's unmodified code.  The
fixture stores the frames (inputs) and the reference's outputs in canonical,
order-free form.  No source is copied.
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

import make_s1_golden as s1g  # noqa: E402

CONFIGS = {
    "scannet": dict(mask_visible_threshold=0.3, undersegment_filter_threshold=0.3,
                    view_consensus_threshold=0.9, contained_threshold=0.8),
    "scannetpp": dict(mask_visible_threshold=0.4, undersegment_filter_threshold=0.2,
                      view_consensus_threshold=1, contained_threshold=0.9),
}


class FrameDataset:
    """The dataset methods the path reads (dataset/scannet.py:34-73), over arrays."""

    def __init__(self, frames, frame_ids, intrinsic_factory):
        self.fr = frames
        self.col = {fid: c for c, fid in enumerate(frame_ids)}
        self.mk = intrinsic_factory

    def get_intrinsics(self, frame_id):
        return self.mk(*self.fr.intrinsics[self.col[frame_id]])

    def get_extrinsic(self, frame_id):
        return self.fr.poses[self.col[frame_id]].copy()

    def get_depth(self, frame_id):
        return self.fr.depth[self.col[frame_id]].copy()

    def get_segmentation(self, frame_id, align_with_depth=False):
        return self.fr.seg[self.col[frame_id]].copy()


def canonical_nodes(nodes, key, prefix):
    out = {}
    mo, mi, vfb, co, ci, po, pi_, info, so, si = [0], [], [], [0], [], [0], [], [], [0], []
    for n in nodes:
        ks = sorted(key(f, m) for f, m in n.mask_list)
        mi.extend(ks); mo.append(len(mi))
        vfb.append(np.packbits(np.asarray(n.visible_frame.cpu() if hasattr(n.visible_frame, "cpu") else n.visible_frame) > 0))
        c = np.nonzero(np.asarray(n.contained_mask.cpu() if hasattr(n.contained_mask, "cpu") else n.contained_mask) > 0)[0]
        ci.extend(c.tolist()); co.append(len(ci))
        p = sorted(int(x) for x in n.point_ids)
        pi_.extend(p); po.append(len(pi_))
        info.append(tuple(n.node_info))
        s = sorted(tuple(x) for x in n.son_node_info) if n.son_node_info else []
        si.extend([x[1] for x in s]); so.append(len(si))
    out[prefix + "mask_off"], out[prefix + "mask_idx"] = np.array(mo, np.int64), np.array(mi, np.int32)
    out[prefix + "vf_bits"] = np.array(vfb, np.uint8).reshape(len(nodes), -1)
    out[prefix + "c_off"], out[prefix + "c_idx"] = np.array(co, np.int64), np.array(ci, np.int32)
    out[prefix + "pt_off"], out[prefix + "pt_idx"] = np.array(po, np.int64), np.array(pi_, np.int32)
    out[prefix + "node_info"] = np.array(info, np.int32).reshape(-1, 2)
    out[prefix + "son_off"], out[prefix + "son_idx"] = np.array(so, np.int64), np.array(si, np.int32)
    return out


def canonical_outputs(nodes0, thr, mpc, pfm, objects, frame_ids):
    col = {fid: c for c, fid in enumerate(frame_ids)}
    keys = sorted(mpc.keys(), key=lambda k: (col[type(frame_ids[0])(k.rsplit("_", 1)[0])]
                                            if not isinstance(frame_ids[0], str) else col[k.rsplit("_", 1)[0]],
                                            int(k.rsplit("_", 1)[1])))
    kidx = {k: i for i, k in enumerate(keys)}

    def key(f, m):
        return kidx[f"{f}_{m}"]

    out = {}
    out["mpc_col"] = np.array([col[type(frame_ids[0])(k.rsplit("_", 1)[0])] if not isinstance(frame_ids[0], str)
                               else col[k.rsplit("_", 1)[0]] for k in keys], np.int32)
    out["mpc_label"] = np.array([int(k.rsplit("_", 1)[1]) for k in keys], np.int32)
    mo, mi = [0], []
    for k in keys:
        mi.extend(sorted(int(x) for x in mpc[k])); mo.append(len(mi))
    out["mpc_off"], out["mpc_idx"] = np.array(mo, np.int64), np.array(mi, np.int32)
    out["thr_value"] = np.array([float(t) for t in thr], np.float32)
    out["thr_is_int"] = np.array([isinstance(t, int) for t in thr], bool)
    out["pfm_bits"] = np.packbits(np.asarray(pfm, bool), axis=1)
    out.update(canonical_nodes(nodes0, key, "n0_"))
    out.update(canonical_nodes(objects, key, "obj_"))
    return out


def run_reference(frames, frame_ids, cfg_name):
    mb, torch = s1g._import_reference()
    os.environ["TQDM_DISABLE"] = "1"
    from graph import construction, iterative_clustering  # noqa: E402
    assert construction.frame_backprojection is mb.frame_backprojection
    ds = FrameDataset(frames, frame_ids, s1g._Intrinsic)
    args = SimpleNamespace(debug=False, **CONFIGS[cfg_name])
    nodes, thr, mpc, pfm = construction.mask_graph_construction(args, frames.scene_points, list(frame_ids), ds)
    objects = iterative_clustering.iterative_clustering(list(nodes), thr, args.view_consensus_threshold, False)
    return canonical_outputs(nodes, thr, mpc, pfm, objects, list(frame_ids))


def save(name, frames, frame_ids, cfg_name):
    ref = run_reference(frames, frame_ids, cfg_name)
    fid = np.array(frame_ids)
    inp = dict(in_scene=frames.scene_points, in_depth=frames.depth, in_seg=frames.seg,
               in_intrinsics=frames.intrinsics, in_poses=frames.poses, in_frame_ids=fid,
               cfg=np.array([CONFIGS[cfg_name][k] for k in ("mask_visible_threshold", "undersegment_filter_threshold",
                                                            "view_consensus_threshold", "contained_threshold")]),
               cfg_ct_is_int=np.array(isinstance(CONFIGS[cfg_name]["view_consensus_threshold"], int)))
    path = os.path.join(HERE, f"api_{name}.npz")
    np.savez_compressed(path, **inp, **ref)
    print(f"api_{name}: masks={len(ref['mpc_col'])} nodes0={len(ref['n0_node_info'])} thr={ref['thr_value'].tolist()} "
          f"objects={len(ref['obj_node_info'])} -> {os.path.getsize(path) / 1e6:.2f} MB")


def main():
    from maskclustering_amd.synthetic_frames import make_frames_shape
    fr = make_frames_shape("small", seed=4)
    save("small_scannet", fr, [int(x) for x in np.arange(0, 10 * fr.num_frames, 10)], "scannet")
    fr2 = make_frames_shape("small", seed=6, num_frames=12, p_split=0.15, p_merge=0.1)
    save("small_scannetpp", fr2, [f"{i:05d}" for i in range(fr2.num_frames)], "scannetpp")


if __name__ == "__main__":
    main()
