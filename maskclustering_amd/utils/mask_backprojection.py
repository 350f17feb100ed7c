"""Drop-in for the reference's ``utils/mask_backprojection.py`` (S1).

Same names, constants, arguments, return shapes and error behaviour as the
reference; the work runs in libmcgraph's HIP kernels (``mc_backproject``):

* ``turn_mask_to_point(dataset, scene_points, mask_image, frame_id)``
  (reference :70-151) -> ``(mask_info, valid_mask_ids, frame_point_ids)``;
  ``({}, [], set())`` for a pose with inf (:73-74), ``({}, [], [])`` when no
  mask survives (:121-122); IndexError for a depth pixel equal to DEPTH_TRUNC
  (the reference's failure at :100).
* ``frame_backprojection(dataset, scene_points, frame_id)`` (:154-156).
* ``get_depth_mask`` and ``crop_scene_points`` (:42-45, :48-67) are small
  torch helpers of the reference kept for callers that use them directly.

Mask ids are ``np.uint8`` keys in ascending order, like the reference's
``ids = torch.unique(...).cpu().numpy()`` (:77-78); each value is the set of
scene-point ids (:148).
"""
from __future__ import annotations

import numpy as np

from .. import _device
from .._native import MC_ERR_INVALID, McError, bp_params

COVERAGE_THRESHOLD = 0.3
DISTANCE_THRESHOLD = 0.01
FEW_POINTS_THRESHOLD = 25
DEPTH_TRUNC = 20
BBOX_EXPAND = 0.1


def params():
    """The reference's S1 constants as mc_bp_params (module values, so a caller that
    changes them the way the reference's users edit the file is followed)."""
    return bp_params(depth_trunc=float(DEPTH_TRUNC), voxel_size=float(DISTANCE_THRESHOLD),
                     ball_radius=float(DISTANCE_THRESHOLD), coverage_threshold=float(COVERAGE_THRESHOLD),
                     few_points=int(FEW_POINTS_THRESHOLD))


def get_depth_mask(depth):
    import torch
    depth_tensor = torch.from_numpy(depth)
    if torch.cuda.is_available():
        depth_tensor = depth_tensor.cuda()
    return torch.logical_and(depth_tensor > 0, depth_tensor <= DEPTH_TRUNC).reshape(-1)


def crop_scene_points(mask_points, scene_points):
    import torch
    lo = mask_points.min(dim=0).values
    hi = mask_points.max(dim=0).values
    sel = ((scene_points > lo) & (scene_points < hi)).all(dim=1)
    ids = torch.where(sel)[0]
    return scene_points[ids], ids


def _run_frames(scene_points, depth, seg, K, T):
    ctx = _device.context()
    _device.set_scene_points(scene_points)
    try:
        ctx.backproject(depth, seg, K, T, params())
    except McError as e:
        if e.code == MC_ERR_INVALID and "depth_trunc" in str(e):
            raise IndexError(str(e)) from e
        raise
    return ctx.bp_masks()


def turn_mask_to_point(dataset, scene_points, mask_image, frame_id):
    K = _device.intrinsics_tuple(dataset.get_intrinsics(frame_id))
    T = np.asarray(dataset.get_extrinsic(frame_id), np.float64).reshape(4, 4)
    if np.sum(np.isinf(T)) > 0:
        return {}, [], set()
    depth = np.asarray(dataset.get_depth(frame_id), np.float32)
    seg = _device.seg_u8(mask_image).reshape(depth.shape)
    _, lab, off, pts = _run_frames(scene_points, depth[None], seg[None], K[None], T[None])
    if len(lab) == 0:
        return {}, [], []
    mask_info = {}
    frame_point_ids = set()
    for k, mid in enumerate(lab):
        s = set(pts[off[k]:off[k + 1]].tolist())
        mask_info[np.uint8(mid)] = s
        frame_point_ids.update(s)
    return mask_info, [np.uint8(m) for m in lab], list(frame_point_ids)


def frame_backprojection(dataset, scene_points, frame_id):
    mask_image = dataset.get_segmentation(frame_id, align_with_depth=True)
    mask_info, _, frame_point_ids = turn_mask_to_point(dataset, scene_points, mask_image, frame_id)
    return mask_info, frame_point_ids
