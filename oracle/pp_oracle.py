"""CPU restatement of the reference's post-processing compute (TEST INFRASTRUCTURE ONLY).

Only ``tests/`` may import this module, as the checker of the HIP path
(``maskclustering_amd.utils.post_process``); the product never routes through it.

Restates ``utils/post_process.py`` of the reference:

* ``dbscan_process`` (:104-123): Open3D ``cluster_dbscan(eps=0.1, min_points=4)`` on the
  node's points in ``list(node.point_ids)`` order (graph/node.py:45), labels + 1, one object
  per non-empty label class in class order (class 0 = noise);
* ``filter_point`` (:40-101): per object point, frames of the node's visible frames the
  point appears in (pfm) and frames where a mask of the node contains it; keep the point if
  ``n_node / (n_video + 1e-6) > point_filter_threshold``; each mask of the node goes to the
  object it intersects most (first on ties, skipped when it intersects none) with coverage
  ``|mask ∩ object| / |object|``; keep the object if it has a kept point and >= 2 masks;
  bbox = min / max of all the object's points;
* ``merge_overlapping_objects`` (:7-37): the greedy i < j pass with ``judge_bbox_overlay``
  (utils/geometry.py:3-7) and the 0.8 intersection ratios.

The DBSCAN is Open3D's loop taken literally (seeds in index order, expansion from core
points only, a noise point reached later becomes a border point of the reaching cluster)
with nanoflann's ``((dx²+dy²)+dz²) < eps²`` in float64.  Pinned by
``tests/golden/pp_small.npz`` (the reference's own post_process, tests/test_pp_oracle.py).
Pure-Python loops: small cases only.
"""
from __future__ import annotations

import numpy as np


def _neighbours(p: np.ndarray, eps: float):
    e2 = eps * eps
    out = []
    for i0 in range(0, len(p), 1024):
        d = p[i0:i0 + 1024, None, :] - p[None, :, :]
        d2 = (d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2]
        out.extend(np.nonzero(row < e2)[0] for row in d2)
    return out


def dbscan(p: np.ndarray, eps: float, min_points: int) -> np.ndarray:
    """Open3D ClusterDBSCAN labels (-1 = noise), post_process.py:109."""
    n = len(p)
    nbs = _neighbours(p, eps)
    labels = np.full(n, -2, np.int64)
    cl = 0
    queued = np.zeros(n, bool)
    for idx in range(n):
        if labels[idx] != -2:
            continue
        if len(nbs[idx]) < min_points:
            labels[idx] = -1
            continue
        queued[:] = False
        queued[idx] = True
        queue = [j for j in nbs[idx] if not queued[j]]
        queued[queue] = True
        labels[idx] = cl
        h = 0
        while h < len(queue):
            q = queue[h]
            h += 1
            if labels[q] == -1:
                labels[q] = cl
            if labels[q] != -2:
                continue
            labels[q] = cl
            if len(nbs[q]) >= min_points:
                new = [j for j in nbs[q] if not queued[j]]
                queued[new] = True
                queue.extend(new)
        cl += 1
    return labels


def post_process_objects(scene, pfm, mask_pts, mask_col, nodes, point_filter_threshold,
                         eps=0.1, min_points=4, overlapping_ratio=0.8):
    """scene f64 [P,3]; pfm bool [P,F]; mask_pts: list of int arrays (mask -> scene point ids);
    mask_col: frame column of each mask; nodes: list of (mask index list in mask_list order,
    vf bool [F], point id array in list(point_ids) order).
    Returns (point id arrays, mask lists [(mask index, coverage)]) after the merge, in order."""
    tot_pts, tot_box, tot_masks = [], [], []
    for masks, vf, order in nodes:
        if len(masks) < 2:                                    # post_process.py:182
            continue
        order = np.asarray(order, np.int64)
        pts = scene[order]
        lab = dbscan(pts, eps, min_points) + 1                # :109
        count = np.bincount(lab)
        objs = [np.nonzero(lab == c)[0] for c in range(len(count)) if count[c] > 0]   # :115-122
        vcols = np.nonzero(vf)[0]
        n_video = [pfm[order[o]][:, vcols].sum(axis=1) for o in objs]                 # :45-58
        hit = [np.zeros((len(o), len(vcols)), bool) for o in objs]
        obj_masks = [[] for _ in objs]
        for m in masks:                                                               # :68-81
            fpos = np.nonzero(vcols == mask_col[m])[0]
            if len(fpos) == 0:
                raise IndexError("mask frame not among the node's visible frames (post_process.py:69)")
            fpos = fpos[0]
            best, largest, cov = -1, 0, 0.0
            for i, o in enumerate(objs):
                w = np.nonzero(np.isin(order[o], mask_pts[m]))[0]
                hit[i][w, fpos] = True
                if len(w) > largest:
                    best, largest, cov = i, len(w), len(w) / len(o)
            if largest == 0:
                continue
            obj_masks[best].append((m, cov))
        for i, o in enumerate(objs):                                                  # :93-100
            ratio = hit[i].sum(axis=1) / (n_video[i] + 1e-6)
            valid = np.nonzero(ratio > point_filter_threshold)[0]
            if len(valid) == 0 or len(obj_masks[i]) < 2:
                continue
            tot_pts.append(order[o][valid])
            tot_box.append((pts[o].min(axis=0), pts[o].max(axis=0)))
            tot_masks.append(obj_masks[i])
    K = len(tot_pts)
    invalid = np.zeros(K, bool)
    sets = [set(p.tolist()) for p in tot_pts]
    for i in range(K):                                                                # :14-29
        if invalid[i]:
            continue
        for j in range(i + 1, K):
            if invalid[j]:
                continue
            a, b = tot_box[i], tot_box[j]
            if any(a[0][c] > b[1][c] or b[0][c] > a[1][c] for c in range(3)):       # geometry.py:3-7
                continue
            inter = len(sets[i] & sets[j])
            if inter / len(sets[i]) > overlapping_ratio:
                invalid[i] = True
            elif inter / len(sets[j]) > overlapping_ratio:
                invalid[j] = True
    keep = np.nonzero(~invalid)[0]
    return [tot_pts[i] for i in keep], [tot_masks[i] for i in keep]
