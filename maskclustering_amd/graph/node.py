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

    @classmethod
    def level0(cls, src, i, g, graph):
        """init_nodes (construction.py:66-78) node ``i`` (global mask ``g``) of a device graph.  Only
        the graph identity is stored; ``mask_list``, the rows, ``node_info`` and ``point_ids`` (the
        mask's set in ``mask_point_clouds``: the same object, as in the reference) are made from
        ``src`` (a Level0Source) on first read."""
        n = cls.__new__(cls)
        d = n.__dict__
        d["_graph"] = graph
        d["_level0"] = i
        d["_src0"] = (src, g)
        return n

    @classmethod
    def level0_list(cls, src, node0, graph):
        """[level0(src, i, g, graph) for i, g in enumerate(node0)], in one loop (14 k nodes a scene)"""
        new = cls.__new__
        out = []
        ap = out.append
        for i, g in enumerate(node0):
            n = new(cls)
            d = n.__dict__
            d["_graph"] = graph
            d["_level0"] = i
            d["_src0"] = (src, g)
            ap(n)
        return out

    def __getattr__(self, name):
        d = self.__dict__
        if name not in _LAZY0 or "_src0" not in d:
            raise AttributeError(f"'Node' object has no attribute '{name}'")
        src, g = d["_src0"]
        v = d[name] = _lazy0(src, g, d["_level0"], name)
        return v

    @classmethod
    def compact_lazy_points(cls, mask_list, vf_bool, contained_ids, num_masks, point_array, node_info, son_node_info,
                            ordered=False):
        """compact() whose ``point_ids`` set is made from ``point_array`` on first read: the device's
        sorted ids (a plain set), or with ``ordered`` the reference's iteration order of the set
        (mc_setorder_replay; a RefOrderSet that iterates in that order)"""
        n = cls.compact(mask_list, vf_bool, contained_ids, num_masks, None, node_info, son_node_info)
        del n.__dict__["_point_ids"]
        n.__dict__["_pts_arr"] = point_array
        n.__dict__["_pts_ordered"] = bool(ordered)
        return n

    @property
    def point_ids(self):
        d = self.__dict__
        if "_point_ids" not in d:
            if "_src0" in d:
                src, g = d["_src0"]
                d["_point_ids"] = src.mpc.original(src.keys[g])
            elif "_pts_arr" in d:
                a = d.pop("_pts_arr").tolist()
                d["_point_ids"] = RefOrderSet(a) if d.pop("_pts_ordered", False) else set(a)
        return d.get("_point_ids")

    def point_order(self) -> np.ndarray:
        """np.int64 ids in list(self.point_ids) order, without making the set when it is still the
        ordered array the clustering returned"""
        d = self.__dict__
        if "_point_ids" not in d and d.get("_pts_ordered") and "_pts_arr" in d:
            return np.asarray(d["_pts_arr"], np.int64)
        p = self.point_ids
        return np.fromiter(p, np.int64, count=len(p))

    @point_ids.setter
    def point_ids(self, v):
        self.__dict__["_point_ids"] = v

    @property
    def visible_frame(self):
        if self._visible_frame is None:
            self._visible_frame = _device_tensor(self._vf.astype(np.float32))
        return self._visible_frame

    @visible_frame.setter
    def visible_frame(self, v):
        self._visible_frame = v
        self._vf = None
        _touch(self)

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
        _touch(self)

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
        point_ids = self.point_order().tolist()
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


class RefOrderSet(set):
    """A set that iterates in a given order: the order CPython's table gives the reference's own
    set of the same contents and history (graph/node.py:35, restated by mc_setorder_replay), so that
    ``list(node.point_ids)`` (graph/node.py:45, utils/post_process.py:185), ``for`` loops and
    np.fromiter see the reference's order.  Contents, ``len``, ``in`` and the set algebra are the
    plain set's; any in-place change drops the order (iteration is then the table's own)."""

    __slots__ = ("_order",)

    def __init__(self, order=()):
        order = list(order)
        super().__init__(order)
        self._order = order if len(order) == len(self) else None

    def __iter__(self):
        o = self._order
        return iter(o) if o is not None else set.__iter__(self)


def _dropping_order(name):
    base = getattr(set, name)

    def f(self, *a, **kw):
        self._order = None
        return base(self, *a, **kw)
    f.__name__ = name
    return f


for _n in ("add", "discard", "remove", "pop", "clear", "update", "difference_update", "intersection_update",
           "symmetric_difference_update", "__ior__", "__iand__", "__isub__", "__ixor__"):
    setattr(RefOrderSet, _n, _dropping_order(_n))


class Level0Source:
    """The arrays level-0 nodes of one device graph are made from: per global mask its
    (frame_id, mask_id), mask_point_clouds key, visible-frame row and contained ids."""

    def __init__(self, gl, keys, vf, c_off, c_idx, num_masks, mpc):
        self.gl, self.keys, self.vf, self.c_off, self.c_idx = gl, keys, vf, c_off, c_idx
        self.M, self.mpc = num_masks, mpc


def _touch(node):
    """A level-0 node's visibility or containment replaced by the caller: its device graph no longer
    describes the node list, so the S6 fast path must not be taken (iterative_clustering._fast_path)."""
    g = node.__dict__.get("_graph")
    if g is not None:
        g.touched = True


_LAZY0 = ("mask_list", "_vf", "_cids", "_M", "_visible_frame", "_contained_mask", "node_info", "son_node_info")


def _lazy0(src, g, i, k):
    if k == "mask_list":
        return [src.gl[g]]
    if k == "_vf":
        return src.vf[g]
    if k == "_cids":
        return src.c_idx[src.c_off[g]:src.c_off[g + 1]]
    if k == "_M":
        return src.M
    if k == "node_info":
        return (0, i)
    return None  # _visible_frame, _contained_mask, son_node_info


def level0_masks(node):
    """node.mask_list, without making the attribute of an untouched level-0 node"""
    d = node.__dict__
    ml = d.get("mask_list")
    if ml is None and "_src0" in d:
        src, g = d["_src0"]
        return (src.gl[g],)
    return node.mask_list


def _np(t):
    if hasattr(t, "detach"):
        return t.detach().cpu().numpy()
    return np.asarray(t)
