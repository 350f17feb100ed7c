"""Generate golden fixtures by running the REFERENCE graph stages (S2-S6).

Run ONLY in the build container, where /root/reference exists:

    python tests/golden/make_golden.py

It imports the reference's own ``graph/construction.py`` and
``graph/iterative_clustering.py`` unmodified: the
absent third-party modules (open3d, pytorch3d, cv2) are registered as empty
stubs, ``Tensor.cuda`` is the identity (CPU torch), and
``graph.construction.frame_backprojection`` is replaced by a lookup into the
synthetic per-frame mask sets — i.e. the S1 output is supplied as data.

Every output written here is data (inputs and the reference's outputs); no
reference source is copied.  The fixtures pin, per scene:
  * S2  ``build_point_in_mask_matrix``  (construction.py:22-64)
  * S3  ``process_masks``               (construction.py:137-170)
  * S4  ``get_observer_num_thresholds`` (construction.py:80-96)
  * S5  ``init_nodes``                  (construction.py:66-78)
  * S6  ``iterative_clustering``        (iterative_clustering.py:36-43), with
        the partition of every iteration captured around
        ``cluster_into_new_nodes`` (iterative_clustering.py:5-10).
"""
from __future__ import annotations

import os
import sys
import types
from types import SimpleNamespace

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"


def _import_reference():
    sys.dont_write_bytecode = True  # the reference tree is read-only
    for n in ["open3d", "pytorch3d", "pytorch3d.ops", "cv2"]:
        sys.modules.setdefault(n, types.ModuleType(n))
    sys.modules["pytorch3d.ops"].ball_query = None
    os.environ["TQDM_DISABLE"] = "1"
    import torch
    torch.Tensor.cuda = lambda self, *a, **k: self
    if REF not in sys.path:
        sys.path.insert(0, REF)
    from graph import construction, iterative_clustering  # noqa: E402
    import networkx as nx  # noqa: E402
    return construction, iterative_clustering, nx, torch


CONFIGS = {
    # configs/scannet.json, configs/scannetpp.json, configs/tasmap.json
    "scannet": dict(mask_visible_threshold=0.3, undersegment_filter_threshold=0.3,
                    view_consensus_threshold=0.9, contained_threshold=0.8),
    "scannetpp": dict(mask_visible_threshold=0.4, undersegment_filter_threshold=0.2,
                      view_consensus_threshold=1, contained_threshold=0.9),
    "tasmap": dict(mask_visible_threshold=0.2, undersegment_filter_threshold=0.1,
                   view_consensus_threshold=0.9, contained_threshold=0.8),
}


def edge_case_scene():
    """Hand-shaped edge cases on top of a tiny scene:
    gaps in mask ids (incl. 255), a frame whose only mask is empty (frame
    skipped, construction.py:50-51), an empty mask next to non-empty ones
    (kept, all-boundary → under-segmented), a frame with no masks, a mask
    made only of boundary points, and > 500-point masks (visibility escape
    construction.py:119)."""
    sys.path.insert(0, REPO)
    from maskclustering_amd.synthetic import make_scene, SceneMasks
    base = make_scene(4000, 20, 12, 0.15, seed=7, p_split=0.15, p_merge=0.1, p_steal=0.2)
    frames = [[] for _ in range(base.num_frames + 3)]
    for g in range(base.num_masks):
        c = int(base.mask_col[g])
        frames[c].append((int(base.mask_label[g]), base.mask_points(g).copy()))
    rng = np.random.default_rng(3)
    # relabel ids with gaps, keep ascending order
    for c, masks in enumerate(frames):
        if not masks:
            continue
        ids = np.sort(rng.choice(np.arange(1, 256), size=len(masks), replace=False))
        if c == 2:
            ids[-1] = 255
        frames[c] = [(int(i), pts) for i, (_, pts) in zip(ids, masks)]
    F0 = base.num_frames
    # frame F0: only an empty mask -> empty union -> frame skipped entirely
    frames[F0] = [(4, np.zeros(0, np.int32))]
    # frame F0+1: an empty mask next to a big one and a boundary-only mask
    big = np.arange(0, 900, dtype=np.int32)
    frames[F0 + 1] = [(1, np.zeros(0, np.int32)), (2, big), (9, big[:40].copy())]
    # frame F0+2: no masks at all (stays an all-zero column)
    frames[F0 + 2] = []
    # another view of the big region, so the >=500 escape gets exercised
    frames[3].append((256 - 1 if all(l != 255 for l, _ in frames[3]) else 254,
                      np.arange(100, 1300, dtype=np.int32)))
    frames[3].sort(key=lambda t: t[0])
    return SceneMasks.from_frame_lists(base.num_points, frames)


def run_reference(scene, cfg_name, frame_ids):
    construction, iterative_clustering, nx, torch = _import_reference()
    per_frame = scene.per_frame_dicts(frame_ids)
    construction.frame_backprojection = lambda ds, sp, fid: (
        per_frame[fid], list(set().union(*per_frame[fid].values())) if per_frame[fid] else [])
    args = SimpleNamespace(debug=False, **CONFIGS[cfg_name])
    scene_points = np.zeros((scene.num_points, 3), dtype=np.float64)
    frame_list = list(frame_ids)

    boundary, pim, mpc, pfm, gl = construction.build_point_in_mask_matrix(args, scene_points, frame_list, None)
    vf, cm, us = construction.process_masks(frame_list, gl, pim, boundary, mpc, args)
    thr = construction.get_observer_num_thresholds(vf)
    nodes = construction.init_nodes(gl, vf, cm, us, mpc)

    # capture partitions per iteration
    partitions, edge_counts, edge_lists = [], [], []
    orig_cluster = iterative_clustering.cluster_into_new_nodes
    orig_update = iterative_clustering.update_graph

    def update_wrap(nodes_, thr_, ct_):
        G = orig_update(nodes_, thr_, ct_)
        edge_counts.append(G.number_of_edges())
        e = np.array(sorted((min(a, b), max(a, b)) for a, b in G.edges()), dtype=np.int32).reshape(-1, 2)
        edge_lists.append(e)
        return G

    def cluster_wrap(iteration, old_nodes, graph):
        labels = np.full(len(old_nodes), -1, dtype=np.int32)
        for k, comp in enumerate(nx.connected_components(graph)):
            labels[list(comp)] = k
        partitions.append(labels)
        return orig_cluster(iteration, old_nodes, graph)

    iterative_clustering.update_graph = update_wrap
    iterative_clustering.cluster_into_new_nodes = cluster_wrap
    try:
        objects = iterative_clustering.iterative_clustering(nodes, thr, args.view_consensus_threshold, False)
    finally:
        iterative_clustering.update_graph = orig_update
        iterative_clustering.cluster_into_new_nodes = orig_cluster

    # ---- canonicalise -------------------------------------------------------------
    key_to_g = {(fid, int(mid)): g for g, (fid, mid) in enumerate(gl)}
    col_of = {fid: c for c, fid in enumerate(frame_list)}
    out = {}
    out["gl_col"] = np.array([col_of[f] for f, _ in gl], dtype=np.int32)
    out["gl_label"] = np.array([int(m) for _, m in gl], dtype=np.int32)
    out["boundary"] = np.array(sorted(boundary), dtype=np.int32)
    nzp, nzc = np.nonzero(pim)
    out["pim_p"], out["pim_c"], out["pim_v"] = nzp.astype(np.int32), nzc.astype(np.int32), pim[nzp, nzc].astype(np.int32)
    out["pfm_bits"] = np.packbits(pfm, axis=1)
    vfn = vf.numpy() if hasattr(vf, "numpy") else np.asarray(vf)
    cmn = cm.numpy() if hasattr(cm, "numpy") else np.asarray(cm)
    out["vf_bits"] = np.packbits(vfn > 0, axis=1)
    r, c = np.nonzero(cmn)
    out["c_row"], out["c_col"] = r.astype(np.int32), c.astype(np.int32)
    out["undersegment"] = np.array(us, dtype=np.int32)
    out["thr_value"] = np.array([float(t) for t in thr], dtype=np.float32)
    out["thr_is_int"] = np.array([isinstance(t, int) for t in thr], dtype=np.bool_)
    out["thr_is_f32"] = np.array([isinstance(t, np.float32) for t in thr], dtype=np.bool_)
    out["node0_g"] = np.array([key_to_g[(n.mask_list[0][0], int(n.mask_list[0][1]))] for n in nodes], dtype=np.int32)
    out["num_iters"] = np.array(len(partitions), dtype=np.int32)
    for t, lab in enumerate(partitions):
        out[f"part_{t}"] = lab
        out[f"edges_{t}"] = edge_lists[t]
    out["edge_counts"] = np.array(edge_counts, dtype=np.int64)
    # final objects, canonical (order-free inside a node: SURVEY App. A.7)
    fm_off, fm_idx, fp_off, fp_idx, fv_bits, fc_off, fc_idx, f_son = [0], [], [0], [], [], [0], [], []
    for node in objects:
        gs = sorted(key_to_g[(f, int(m))] for f, m in node.mask_list)
        fm_idx.extend(gs); fm_off.append(len(fm_idx))
        pts = sorted(int(p) for p in node.point_ids)
        fp_idx.extend(pts); fp_off.append(len(fp_idx))
        fv_bits.append(np.packbits(np.asarray(node.visible_frame) > 0))
        cc = np.nonzero(np.asarray(node.contained_mask) > 0)[0]
        fc_idx.extend(cc.tolist()); fc_off.append(len(fc_idx))
        f_son.append(sorted(j for _, j in node.son_node_info) if node.son_node_info else [])
    out["obj_mask_off"], out["obj_mask_idx"] = np.array(fm_off, np.int64), np.array(fm_idx, np.int32)
    out["obj_pt_off"], out["obj_pt_idx"] = np.array(fp_off, np.int64), np.array(fp_idx, np.int32)
    out["obj_vf_bits"] = np.array(fv_bits, dtype=np.uint8).reshape(len(objects), -1)
    out["obj_c_off"], out["obj_c_idx"] = np.array(fc_off, np.int64), np.array(fc_idx, np.int32)
    out["obj_node_info"] = np.array([n.node_info for n in objects], dtype=np.int32).reshape(-1, 2)
    so = np.zeros(len(f_son) + 1, np.int64)
    so[1:] = np.cumsum([len(s) for s in f_son])
    out["obj_son_off"], out["obj_son_idx"] = so, np.array([j for s in f_son for j in s], dtype=np.int32)
    return out


def save_case(name, scene, cfg_name, frame_ids):
    ref = run_reference(scene, cfg_name, frame_ids)
    inputs = dict(
        in_num_points=np.array(scene.num_points, np.int64),
        in_num_frames=np.array(scene.num_frames, np.int64),
        in_mask_col=scene.mask_col, in_mask_label=scene.mask_label,
        in_mask_off=scene.mask_off, in_mask_pts=scene.mask_pts,
        cfg=np.array([CONFIGS[cfg_name][k] for k in ("mask_visible_threshold", "undersegment_filter_threshold",
                                                     "view_consensus_threshold", "contained_threshold")], np.float64),
        cfg_ct_is_int=np.array(isinstance(CONFIGS[cfg_name]["view_consensus_threshold"], int)),
    )
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **inputs, **ref)
    print(f"{name}: M={len(ref['gl_col'])} U={len(ref['undersegment'])} thr={ref['thr_value'].tolist()} "
          f"iters={int(ref['num_iters'])} objects={len(ref['obj_mask_off']) - 1} "
          f"-> {os.path.getsize(path) / 1e6:.2f} MB")


def save_unit_cases():
    """Direct calls of two reference functions on crafted inputs:
    * get_observer_num_thresholds (construction.py:80-96) on small random VF
      matrices, so that percentiles land between distinct order statistics
      (fractional thresholds, numpy-2 float32 lerp) and on ones that break early;
    * update_graph (iterative_clustering.py:13-33) on crafted node vectors whose
      supporter/observer ratios sit exactly on the 0.9 / 1.0 thresholds."""
    construction, iterative_clustering, nx, torch = _import_reference()
    rng = np.random.default_rng(11)
    out = {}
    n_thr = 0
    for case in range(60):
        M = int(rng.integers(2, 40))
        F = int(rng.integers(2, 30))
        dens = rng.uniform(0.05, 0.9)
        vf = (rng.random((M, F)) < dens).astype(np.float32)
        vft = torch.from_numpy(vf)
        try:
            thr = construction.get_observer_num_thresholds(vft)
            err = 0
        except IndexError:
            thr, err = [], 1
        out[f"thr_vf_{n_thr}"] = np.packbits(vf > 0, axis=1)
        out[f"thr_F_{n_thr}"] = np.array(F)
        out[f"thr_err_{n_thr}"] = np.array(err)
        out[f"thr_val_{n_thr}"] = np.array([float(t) for t in thr], np.float32)
        out[f"thr_isint_{n_thr}"] = np.array([isinstance(t, int) for t in thr], np.bool_)
        n_thr += 1
    out["thr_cases"] = np.array(n_thr)

    # crafted update_graph: node k has visible frames / contained masks chosen so
    # pairs (0,1): O=10,S=9; (2,3): O=1,S=1; (4,5): O=20,S=18; (6,7): O=3,S=2 (0.667)
    F, M = 40, 60
    specs = [(10, 9), (1, 1), (20, 18), (3, 2), (7, 7), (30, 27), (11, 10)]
    vfs, cms = [], []
    for i, (o, s) in enumerate(specs):
        a = np.zeros(F, np.float32); a[:o] = 1
        b = np.zeros(F, np.float32); b[:o] = 1
        ca = np.zeros(M, np.float32); ca[:s] = 1; ca[40 + i] = 1
        cb = np.zeros(M, np.float32); cb[:s] = 1; cb[50 + (i % 10)] = 1
        vfs += [a, b]; cms += [ca, cb]
    from graph.node import Node
    nodes = [Node([(0, k)], torch.from_numpy(v), torch.from_numpy(c), set(), (0, k), None)
             for k, (v, c) in enumerate(zip(vfs, cms))]
    out["ug_vf"] = np.array(vfs); out["ug_cm"] = np.array(cms)
    for ct_name, ct in (("0p9", 0.9), ("1", 1), ("0p8", 0.8)):
        for thr_name, thr in (("1", 1), ("2p5", np.float32(2.5)), ("10", np.float32(10.0))):
            G = iterative_clustering.update_graph(nodes, thr, ct)
            A = nx.to_numpy_array(G, nodelist=range(len(nodes)), dtype=np.int8) > 0
            out[f"ug_A_{ct_name}_{thr_name}"] = np.packbits(A, axis=1)
    path = os.path.join(HERE, "unit_cases.npz")
    np.savez_compressed(path, **out)
    print(f"unit_cases: {n_thr} threshold cases -> {os.path.getsize(path) / 1e6:.2f} MB")


def main():
    sys.path.insert(0, REPO)
    save_unit_cases()
    from maskclustering_amd.synthetic import make_shape, make_scene
    tiny = make_shape("tiny", seed=0)
    save_case("tiny_scannet", tiny, "scannet", [int(x) for x in np.arange(0, 10 * tiny.num_frames, 10)])
    edge = edge_case_scene()
    save_case("edge_scannet", edge, "scannet", [f"{i:08d}" for i in range(edge.num_frames)])
    save_case("edge_scannetpp", edge, "scannetpp", list(range(edge.num_frames)))
    c1 = make_shape("c1", seed=0)
    save_case("c1_scannet", c1, "scannet", list(np.arange(0, 10 * c1.num_frames, 10)))
    c1b = make_shape("c1", seed=1, p_split=0.12, p_steal=0.05)
    save_case("c1_scannetpp", c1b, "scannetpp", list(range(c1b.num_frames)))
    c1c = make_scene(12000, 80, 150, 0.06, seed=2, p_merge=0.1)
    save_case("mid_tasmap", c1c, "tasmap", [f"{i:05d}" for i in range(c1c.num_frames)])


if __name__ == "__main__":
    main()
