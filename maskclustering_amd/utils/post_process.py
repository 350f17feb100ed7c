"""Drop-in for the reference's ``utils/post_process.py``.

``post_process(dataset, node_list, mask_point_clouds, scene_points, point_frame_matrix,
frame_list, args)`` keeps the reference's signature and files (post_process.py:173-195).
Its compute runs on the device in one C-ABI call (``mc_pp_run``, include/mcgraph.h):

* ``dbscan_process`` (:104-123): DBSCAN(eps 0.1, min_points 4) of every node's points at once,
  one workgroup per node on a hashed grid, in ``list(node.point_ids)`` order (graph/node.py:45),
  which is what fixes Open3D's label numbering;
* ``filter_point`` (:40-101): detection ratios from the packed point-frame bits and the node's
  masks, mask -> object assignment and coverage, per-object kept points and bboxes;
* ``merge_overlapping_objects`` (:7-37): pairwise intersections from a point -> object index,
  the bbox / ratio decision of every pair, and the greedy pass in one workgroup.

The host packs the inputs (mask table from ``mask_point_clouds``, point orders, bit rows) and
rebuilds the reference's lists.  When ``mask_point_clouds`` is the one this package's
``mask_graph_construction`` returned (graph.construction.MaskPointClouds, unmodified), the
device gets the CSR rows the sets were made from instead of a re-read of every set; ``export`` (:148-170) writes the same files as the reference.
Errors follow the reference: a mask missing from ``mask_point_clouds`` raises KeyError (:70), a
mask whose frame is not among its node's visible frames raises IndexError (:69).
"""
from __future__ import annotations

import os

import numpy as np

from .. import _device
from .._hostutil import no_gc
from .._native import PPParams


def _host(x):
    if hasattr(x, "detach"):
        return x.detach().cpu().numpy()
    return np.asarray(x)


def _bits(rows_bool: np.ndarray, F: int) -> np.ndarray:
    """bool [R, F] -> little-endian u64 words [R, ceil(F/64)] (bit c of word c // 64 = column c)."""
    FW = (F + 63) // 64
    b = np.packbits(np.asarray(rows_bool, bool).reshape(-1, F), axis=1, bitorder="little")
    out = np.zeros((b.shape[0], FW * 8), np.uint8)
    out[:, :b.shape[1]] = b
    return out.view("<u8")


def _visible(node) -> np.ndarray:
    if hasattr(node, "visible_bool"):
        return np.asarray(node.visible_bool(), bool)
    return _host(node.visible_frame) > 0


def _order(n):
    """np.int64 ids in list(n.point_ids) order (node.py:45)"""
    po = getattr(n, "point_order", None)
    return po() if po is not None else np.fromiter(n.point_ids, np.int64, count=len(n.point_ids))


def _bulk_columns(nodes, vfs, fcol, F):
    """(frame column of every mask of every node, the (frame, mask) pairs), flattened in node order,
    when each mask's frame is visible to its node (the usual case, :67-69 then picks that column); None
    when any is not, for the per-node walk"""
    if not nodes or any(len(v) != F for v in vfs):
        return None
    mls = [n.mask_list for n in nodes]
    flat = [t for ml in mls for t in ml]
    cols = np.array([fcol.get(f, -1) for f, _ in flat], np.int64)
    if len(cols) and cols.min() < 0:
        return None
    owner = np.repeat(np.arange(len(mls)), np.fromiter(map(len, mls), np.int64, count=len(mls)))
    if not np.stack(vfs)[owner, cols].all():
        return None
    return cols, flat


def post_process_objects(node_list, mask_point_clouds, scene_points, point_frame_matrix, frame_list,
                         point_filter_threshold, dbscan_eps=0.1, dbscan_min_points=4, overlapping_ratio=0.8):
    """post_process.py:180-194 on the device: returns (total_point_ids_list, total_mask_list) as the
    reference hands them to export (object point ids int64 in list order; [(frame_id, mask_id,
    coverage)] per object)."""
    with no_gc():
        return _post_process_objects(node_list, mask_point_clouds, scene_points, point_frame_matrix, frame_list,
                                     point_filter_threshold, dbscan_eps, dbscan_min_points, overlapping_ratio)


def _post_process_objects(node_list, mask_point_clouds, scene_points, point_frame_matrix, frame_list,
                          point_filter_threshold, dbscan_eps, dbscan_min_points, overlapping_ratio):
    nodes = [n for n in node_list if len(n.mask_list) >= 2]   # :182
    frame_arr = np.array(frame_list)
    F = len(frame_list)
    table, mask_arrays = {}, []
    q_mask, q_col, q_key, vf_rows, orders = [], [], [], [], []
    csr = getattr(mask_point_clouds, "csr", None)   # rows the drop-in construction made the sets from
    fcol = {}
    for c, fid in enumerate(frame_arr.tolist()):
        fcol.setdefault(fid, c)
    unique_frames = len(fcol) == F

    lazy = csr is not None and hasattr(mask_point_clouds, "is_materialized")
    # no set of the mapping made yet (the drop-in construction's lazy mapping, untouched): every key
    # is served by its CSR row, looked up directly (KeyError for a missing key, as at :70)
    direct = lazy and dict.__len__(mask_point_clouds) == 0
    row_of = csr[0] if direct else None
    q_rows = []

    def add(key):
        if lazy and not mask_point_clouds.is_materialized(key):  # the CSR row serves it: no set made
            if key not in mask_point_clouds:
                raise KeyError(key)
            pts = None
        else:
            pts = mask_point_clouds[key]                          # KeyError as at :70
        table[key] = len(mask_arrays)
        mask_arrays.append(pts)

    vfs = [_visible(n) for n in nodes]
    bulk = _bulk_columns(nodes, vfs, fcol, F) if direct and unique_frames else None
    if bulk is not None:        # every mask's frame visible to its node: one pass, in node order
        cols, q_key = bulk
        q_rows = [row_of[f"{f}_{m}"] for f, m in q_key]         # KeyError as at :70
        q_col = cols.tolist()
        vf_rows = vfs
        orders = [_order(n) for n in nodes]
    for n, vf in zip(nodes if bulk is None else (), vfs):
        ml = n.mask_list
        cols = np.array([fcol.get(f, -1) for f, _ in ml], np.int64) if unique_frames else None
        if cols is not None and (cols >= 0).all() and vf[cols].all():
            keys = [f"{f}_{m}" for f, m in ml]
            if direct:
                q_rows.extend([row_of[k] for k in keys])
            else:
                for key in keys:
                    if key not in table:
                        add(key)
                q_mask.extend([table[k] for k in keys])
            q_col.extend(cols.tolist())
            q_key.extend(ml)
        else:                                                     # per mask, in the reference's order
            vcols = np.nonzero(vf)[0]
            first = {}                                            # frame id -> first visible column (:69)
            for c, fid in zip(vcols.tolist(), frame_arr[vcols].tolist()):
                first.setdefault(fid, c)
            for f, m in ml:
                c = first.get(f)
                if c is None:                                     # :69
                    raise IndexError("index 0 is out of bounds for axis 0 with size 0")
                key = f"{f}_{m}"
                if direct:
                    q_rows.append(row_of[key])
                else:
                    if key not in table:
                        add(key)
                    q_mask.append(table[key])
                q_col.append(c)
                q_key.append((f, m))
        vf_rows.append(vf)
        orders.append(_order(n))
    if not nodes:
        return [], []
    scene = np.ascontiguousarray(_host(scene_points), np.float64).reshape(-1, 3)
    pfm = getattr(point_frame_matrix, "_mc_bits", None)           # construction's packed words
    if pfm is None or point_frame_matrix.flags.writeable or point_frame_matrix.shape[1] != F:
        pfm = _bits(_host(point_frame_matrix), F)
    if direct:
        q_dev = np.asarray(q_rows, np.int64)
        mask_off, mask_pts = csr[1], csr[2]
    else:
        if csr is not None:  # the construction's rows: table entry -> CSR row, no set is re-read
            rows = np.fromiter((csr[0][k] for k in table), np.int64, count=len(table))
            clen = np.diff(csr[1])[rows]
            lens = np.fromiter((len(p) if p is not None else -1 for p in mask_arrays), np.int64, count=len(mask_arrays))
            lens = np.where(lens < 0, clen, lens)
            if not np.array_equal(clen, lens):                    # a set changed in place
                csr = None
                mask_arrays = [p if p is not None else mask_point_clouds[k] for k, p in zip(table, mask_arrays)]
        if csr is not None:
            q_dev = rows[np.asarray(q_mask, np.int64)]
            mask_off, mask_pts = csr[1], csr[2]
        else:
            q_dev = np.asarray(q_mask, np.int64)
            arrs = [np.fromiter(p, np.int64, count=len(p)) for p in mask_arrays]
            mask_off = np.zeros(len(arrs) + 1, np.int64)
            np.cumsum([len(a) for a in arrs], out=mask_off[1:])
            mask_pts = np.concatenate(arrs) if arrs else np.zeros(0, np.int64)
    pt_off = np.zeros(len(nodes) + 1, np.int64)
    np.cumsum([len(o) for o in orders], out=pt_off[1:])
    q_off = np.zeros(len(nodes) + 1, np.int64)
    np.cumsum([len(n.mask_list) for n in nodes], out=q_off[1:])
    pts_all = np.concatenate(orders)
    prm = PPParams(float(dbscan_eps), int(dbscan_min_points), float(point_filter_threshold), float(overlapping_ratio))
    ctx = _device.context()
    ctx.pp_run(prm, scene, pfm, F, mask_off, mask_pts, _bits(np.stack(vf_rows), F), pt_off, pts_all, q_off, q_dev,
               np.array(q_col, np.int32))
    r = ctx.pp_results()
    final = np.nonzero(r["object_state"] == 2)[0]
    ent, onode = r["entry_object"], r["object_node"]
    out_pts = []
    for o, k in zip(final.tolist(), onode[final].tolist()):
        a, b = pt_off[k], pt_off[k + 1]
        out_pts.append(pts_all[a:b][ent[a:b] == o])
    slot = np.full(len(r["object_state"]) + 1, -1, np.int64)
    slot[final] = np.arange(len(final))
    qslot = slot[r["mask_object"]]                                # mask_object -1 -> slot[-1] = -1
    out_masks = [[] for _ in final]
    sel = np.nonzero(qslot >= 0)[0]                               # node order, then mask_list order
    for q, sl, cov in zip(sel.tolist(), qslot[sel].tolist(), r["mask_coverage"][sel].tolist()):
        f, m = q_key[q]
        out_masks[sl].append((f, m, cov))
    return out_pts, out_masks


def find_represent_mask(mask_info_list):
    """post_process.py:126-128: the five masks of largest coverage (sorts the list in place)."""
    mask_info_list.sort(key=lambda x: x[2], reverse=True)
    return mask_info_list[:5]


def export_class_agnostic_mask(args, class_agnostic_mask_list):
    """post_process.py:131-145: data/prediction/<config>_class_agnostic/<seq_name>.npz."""
    os.makedirs(os.path.join("data/prediction", args.config), exist_ok=True)
    n = len(class_agnostic_mask_list)
    out_dir = os.path.join("data/prediction", args.config + "_class_agnostic")
    os.makedirs(out_dir, exist_ok=True)
    np.savez(os.path.join(out_dir, f"{args.seq_name}.npz"), pred_masks=np.stack(class_agnostic_mask_list, axis=1),
             pred_score=np.ones(n), pred_classes=np.zeros(n, dtype=np.int32))


def export(dataset, total_point_ids_list, total_mask_list, args):
    """post_process.py:148-170: binary masks over the scene points + the object dict."""
    P = dataset.get_scene_points().shape[0]
    masks, object_dict = [], {}
    for i, (point_ids, mask_list) in enumerate(zip(total_point_ids_list, total_mask_list)):
        object_dict[i] = {"point_ids": point_ids, "mask_list": mask_list,
                          "repre_mask_list": find_represent_mask(mask_list)}
        m = np.zeros(P, dtype=bool)
        m[list(point_ids)] = True
        masks.append(m)
    export_class_agnostic_mask(args, masks)
    out_dir = os.path.join(dataset.object_dict_dir, args.config)
    os.makedirs(out_dir, exist_ok=True)
    np.save(os.path.join(out_dir, "object_dict.npy"), object_dict, allow_pickle=True)


def post_process(dataset, node_list, mask_point_clouds, scene_points, point_frame_matrix, frame_list, args):
    """post_process.py:173-195."""
    if args.debug:
        print('start exporting')
    pts, masks = post_process_objects(node_list, mask_point_clouds, scene_points, point_frame_matrix, frame_list,
                                      args.point_filter_threshold)
    export(dataset, pts, masks, args)
