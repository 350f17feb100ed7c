"""Drop-in for the reference's ``graph/node.py`` (the cluster record).

``Node(mask_list, visible_frame, contained_mask, point_ids, node_info,
son_node_info)`` has the reference's attributes (graph/node.py:6-21).  Nodes
made by this package's graph construction / clustering hold the visible-frame
row as packed bits and the contained row as sorted mask ids, and materialise
the reference's dense float tensors (``visible_frame`` [F], ``contained_mask``
[M], on the current CUDA device) only when those attributes are read, e.g. by
post_process (utils/post_process.py:84).  Assigning them stores the tensor as
given, as in the reference.
"""
from __future__ import annotations

import numpy as np


def _device_tensor(x):
    import torch
    t = torch.from_numpy(np.ascontiguousarray(x, np.float32))
    return t.cuda() if torch.cuda.is_available() else t


class Node:

    def __init__(self, mask_list, visible_frame, contained_mask, point_ids, node_info, son_node_info):
        self.mask_list = mask_list
        self.visible_frame = visible_frame
        self.contained_mask = contained_mask
        self.point_ids = point_ids
        self.node_info = node_info
        self.son_node_info = son_node_info

    # compact form used by the device path ------------------------------------------------------
    @classmethod
    def compact(cls, mask_list, vf_bool, contained_ids, num_masks, point_ids, node_info, son_node_info):
        n = cls.__new__(cls)
        n.mask_list = mask_list
        n._vf = np.asarray(vf_bool, bool)
        n._cids = np.asarray(contained_ids, np.int32)
        n._M = int(num_masks)
        n._visible_frame = None
        n._contained_mask = None
        n.point_ids = point_ids
        n.node_info = node_info
        n.son_node_info = son_node_info
        return n

    @property
    def visible_frame(self):
        if self._visible_frame is None:
            self._visible_frame = _device_tensor(self._vf.astype(np.float32))
        return self._visible_frame

    @visible_frame.setter
    def visible_frame(self, v):
        self._visible_frame = v
        self._vf = None

    @property
    def contained_mask(self):
        if self._contained_mask is None:
            d = np.zeros(self._M, np.float32)
            d[self._cids] = 1.0
            self._contained_mask = _device_tensor(d)
        return self._contained_mask

    @contained_mask.setter
    def contained_mask(self, v):
        self._contained_mask = v
        self._cids = None

    def visible_bool(self) -> np.ndarray:
        """visible_frame > 0 as a host bool row (no dense tensor round trip when compact)."""
        if getattr(self, "_vf", None) is not None:
            return self._vf
        return _np(self._visible_frame) > 0

    def contained_ids(self) -> np.ndarray:
        if getattr(self, "_cids", None) is not None:
            return self._cids
        return np.nonzero(_np(self._contained_mask) > 0)[0].astype(np.int32)

    def num_masks(self) -> int:
        if getattr(self, "_cids", None) is not None:
            return self._M
        return int(len(self._contained_mask))

    # reference methods -------------------------------------------------------------------------
    @staticmethod
    def create_node_from_list(node_list, node_info):
        """graph/node.py:24-37: OR of the members' rows, concatenated mask lists, union of point sets."""
        mask_list = []
        vf = np.zeros(len(node_list[0].visible_bool()), bool)
        cids = []
        point_ids = set()
        son_node_info = set()
        for node in node_list:
            mask_list += node.mask_list
            vf |= node.visible_bool()
            cids.append(node.contained_ids())
            point_ids = point_ids.union(node.point_ids)
            son_node_info.add(node.node_info)
        c = np.unique(np.concatenate(cids)) if cids else np.zeros(0, np.int32)
        return Node.compact(mask_list, vf, c, node_list[0].num_masks(), point_ids, node_info, son_node_info)

    def get_point_cloud(self, scene_points):
        """graph/node.py:39-49 (an Open3D PointCloud when open3d is importable)."""
        point_ids = list(self.point_ids)
        points = np.asarray(scene_points)[point_ids]
        try:
            import open3d as o3d
            pcld = o3d.geometry.PointCloud()
            pcld.points = o3d.utility.Vector3dVector(points)
        except ImportError:
            class _PointCloud:
                pass
            pcld = _PointCloud()
            pcld.points = points
        return pcld, point_ids


def _np(t):
    if hasattr(t, "detach"):
        return t.detach().cpu().numpy()
    return np.asarray(t)
