"""Drop-in for the reference's ``graph/construction.py`` (S1-S5).

``mask_graph_construction(args, scene_points, frame_list, dataset)`` keeps the
reference's signature and return value (construction.py:7-20):
``(nodes, observer_num_thresholds, mask_point_clouds, point_frame_matrix)``.
Every frame is back-projected and the graph is built on the device in one
pass (mc_backproject + mc_graph_build); the host only stacks the dataset's
per-frame arrays and rebuilds the Python containers the caller reads:

* ``nodes``: one ``Node`` per non-under-segmented mask in global order
  (init_nodes, :66-78), ``node_info = (0, i)``, ``point_ids`` aliasing the
  mask's set in ``mask_point_clouds`` like the reference;
* ``observer_num_thresholds``: ``np.float32`` values or the int 1 (:88-95);
* ``mask_point_clouds``: ``{f"{frame_id}_{mask_id}": set}`` (:57);
* ``point_frame_matrix``: ``np.bool_`` [P, F] (:40,52).

The other public functions of the reference module are provided with the same
signatures (build_point_in_mask_matrix, process_masks, init_nodes,
get_observer_num_thresholds); they run the same device stages.
Errors follow the reference: IndexError for a DEPTH_TRUNC depth pixel and for
an empty observer-count list (np.percentile of an empty array, :89).
"""
from __future__ import annotations

import itertools

import os

import numpy as np

from .. import _device
from .._hostutil import no_gc
from .. import _native
from .._native import MC_ERR_EMPTY_OBSERVERS, MC_ERR_INVALID, McError
from ..pipeline import bits_to_bool, bool_to_bits
from ..utils import mask_backprojection as _mb
from .node import Level0Source, Node

_tokens = itertools.count(1)


class PointFrameMatrix(np.ndarray):
    """point_frame_matrix (construction.py:40,52): the reference's bool [P, F] array, read-only (the
    reference's callers only read it), carrying the packed bits it was unpacked from so that
    utils.post_process hands them to the device without re-packing 60 MB at C2."""

    @classmethod
    def from_bits(cls, words, F):
        a = _native.bits_unpack(words, F).view(cls)
        a._mc_bits = np.ascontiguousarray(words)
        a.flags.writeable = False
        return a

    def __array_finalize__(self, obj):
        self._mc_bits = None  # views / copies / results of operations carry no bits


class GraphHandle:
    """Identifies the device graph a level-0 node list came from (fast S6 path)."""

    def __init__(self, token, num_nodes, num_frames, num_masks, num_points, src=None, node0=None):
        self.token = token
        self.num_nodes = num_nodes
        self.num_frames = num_frames
        self.num_masks = num_masks
        self.num_points = num_points
        self.src = src      # Level0Source of the level-0 nodes
        self.node0 = node0  # global mask of every level-0 node
        self.nodes = ()     # the level-0 Node objects, in order (the fast path checks identity)
        self.touched = False  # set by a node's visible_frame / contained_mask setter


_current = {"token": None}


def _raw_depth_scale(dataset):
    """depth_scale when the dataset hands out its depth PNGs' raw values: an optional
    ``get_depth_raw(frame_id)`` returning the uint16 array that the reference's datasets divide by
    ``depth_scale`` in get_depth (dataset/scannet.py:49-54, scannetpp.py:166-171,
    matterport.py:89-94).  The frames then cross PCIe at 2 bytes per pixel and are divided on the
    device, bit-identical to get_depth's float32.  MASKCLUSTERING_RAW_DEPTH=0:
    always get_depth."""
    if os.environ.get("MASKCLUSTERING_RAW_DEPTH", "1") == "0" or not callable(getattr(dataset, "get_depth_raw", None)):
        return None
    scale = getattr(dataset, "depth_scale", None)
    return float(scale) if scale is not None and float(scale) > 0 else None


def _read_frames(frame_list, dataset, raw_scale=None):
    """the dataset calls of construction.py:47-48 / mask_backprojection.py:71-80, per frame (the
    arrays are handed to the device as they are, no [F,H,W] host stack); raw_scale: the depth
    frames are get_depth_raw's uint16 values"""
    depth, seg, K, T = [], [], [], []
    for frame_id in frame_list:
        if raw_scale is not None:
            d = np.asarray(dataset.get_depth_raw(frame_id))
            if d.dtype != np.uint16:
                raise TypeError("get_depth_raw must return the depth PNG's uint16 values")
            depth.append(np.ascontiguousarray(d))
        else:
            depth.append(np.ascontiguousarray(dataset.get_depth(frame_id), np.float32))
        seg.append(np.ascontiguousarray(_device.seg_u8(dataset.get_segmentation(frame_id, align_with_depth=True))))
        K.append(_device.intrinsics_tuple(dataset.get_intrinsics(frame_id)))
        T.append(np.asarray(dataset.get_extrinsic(frame_id), np.float64).reshape(4, 4))
    if any(d.shape != depth[0].shape or s.shape != depth[0].shape for d, s in zip(depth, seg)):
        raise ValueError("all frames must share one depth / segmentation shape")
    return depth, seg, np.stack(K), np.stack(T)


def _backproject_all(scene_points, frame_list, dataset):
    ctx = _device.context()
    _device.set_scene_points(scene_points)
    if len(frame_list) == 0:
        ctx.backproject(np.zeros((0, 1, 1), np.float32), np.zeros((0, 1, 1), np.uint8), np.zeros((0, 4)),
                        np.zeros((0, 4, 4)), _mb.params())
        return ctx
    raw_scale = _raw_depth_scale(dataset)
    depth, seg, K, T = _read_frames(frame_list, dataset, raw_scale)
    try:
        ctx.backproject_frames(depth, seg, K, T, _mb.params(), depth_scale=raw_scale)
    except McError as e:
        if e.code == MC_ERR_INVALID and "depth_trunc" in str(e):
            raise IndexError(str(e)) from e
        raise
    return ctx


class MaskPointClouds(dict):
    """``{f"{frame_id}_{mask_id}": set}`` exactly as the reference builds it (:57), built lazily: the
    sets are made from the device's CSR rows on first access (one set per mask: 3.7 M Python ints
    at C2 that the graph path itself never reads).  Iteration, ``len``, ``in``, ``keys`` / ``values``
    / ``items`` and every mutator see the full mapping in the reference's insertion order (the
    global mask order).  ``csr`` (key -> row, offsets, point ids) lets utils.post_process hand the
    device the rows instead of re-reading the sets; any mutation of the mapping drops it, and
    post_process checks the sizes of the sets that were materialised."""

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.csr = None
        self._lazy = {}
        self._made = {}
        self._order = None

    @classmethod
    def from_csr(cls, keys, off, pts):
        m = cls()
        m._lazy = {k: g for g, k in enumerate(keys)}  # a repeated key maps to its last row
        m._order = list(dict.fromkeys(keys))          # ... at its first position, as a dict keeps it
        m._off, m._pts = off, pts
        m.csr = (dict(m._lazy), off, pts)
        return m

    def _make(self, k):
        g = self._lazy.pop(k)
        v = self._made[k] = set(self._pts[self._off[g]:self._off[g + 1]].tolist())
        dict.__setitem__(self, k, v)
        return v

    def original(self, k):
        """the set first stored under ``k`` (a level-0 node's point_ids aliases it even after the
        mapping is changed, as in the reference)"""
        v = self._made.get(k)
        if v is None:
            v = self._make(k) if k in self._lazy else self[k]
        return v

    def __missing__(self, k):
        if k in self._lazy:
            return self._make(k)
        raise KeyError(k)

    def is_materialized(self, k):
        return dict.__contains__(self, k)

    def _materialize(self):
        """every set made, dict order = the reference's insertion order"""
        if self._order is None:
            return
        if self._lazy:
            items = [(k, dict.get(self, k) if dict.__contains__(self, k) else None) for k in self._order]
            dict.clear(self)
            for k, v in items:
                if v is None:
                    g = self._lazy.pop(k)
                    v = self._made[k] = set(self._pts[self._off[g]:self._off[g + 1]].tolist())
                dict.__setitem__(self, k, v)
        self._order = None

    def __contains__(self, k):
        return dict.__contains__(self, k) or k in self._lazy

    def __len__(self):
        return dict.__len__(self) + len(self._lazy)

    def __iter__(self):
        self._materialize()
        return dict.__iter__(self)

    def get(self, k, default=None):
        return self[k] if k in self else default

    def _drop(self):
        self._materialize()
        self.csr = None

    def __setitem__(self, k, v):
        self._drop()
        super().__setitem__(k, v)

    def __delitem__(self, k):
        self._drop()
        super().__delitem__(k)

    def __eq__(self, other):
        self._materialize()
        return dict.__eq__(self, other)

    def __ne__(self, other):
        return not self.__eq__(other)

    __hash__ = None

    def __repr__(self):
        self._materialize()
        return dict.__repr__(self)

    def __reduce__(self):
        self._materialize()
        return (dict, (dict(self),))


def _reading(name):
    def f(self, *a, **kw):
        self._materialize()
        return getattr(dict, name)(self, *a, **kw)
    f.__name__ = name
    return f


def _dropping(name):
    def f(self, *a, **kw):
        self._drop()
        return getattr(dict, name)(self, *a, **kw)
    f.__name__ = name
    return f


for _n in ("keys", "values", "items", "copy", "__reversed__"):
    setattr(MaskPointClouds, _n, _reading(_n))
for _n in ("update", "pop", "popitem", "clear", "setdefault"):
    setattr(MaskPointClouds, _n, _dropping(_n))


def _mask_sets(ctx, frame_list):
    col, lab, off, pts = ctx.bp_masks()
    fl = [frame_list[c] for c in col.tolist()]
    gl = list(zip(fl, np.asarray(lab).astype(np.uint8)))          # (frame id, np.uint8 mask id)
    keys = [f"{f}_{m}" for f, m in zip(fl, np.asarray(lab).tolist())]  # ints format as the uint8s do
    return gl, keys, MaskPointClouds.from_csr(keys, np.asarray(off, np.int64), np.asarray(pts))


def _thresholds(thr, isint):
    return [1 if i else np.float32(t) for t, i in zip(thr.tolist(), isint.tolist())]


def _build(args, scene_points, frame_list, dataset):
    _current["token"] = None  # the device graph is about to be replaced
    ctx = _backproject_all(scene_points, frame_list, dataset)
    gl_in, keys_in, mpc = _mask_sets(ctx, frame_list)
    ctx.use_backprojection()
    ctx.build(args.mask_visible_threshold, args.contained_threshold, args.undersegment_filter_threshold)
    gi = ctx.graph_info()
    # frames whose union is empty are skipped (construction.py:50-51): global list = kept input masks
    gidx = ctx.global_masks(gi.num_masks)
    gl = [gl_in[i] for i in gidx.tolist()]
    keys = [keys_in[i] for i in gidx.tolist()]
    return ctx, gi, gl, keys, mpc


def mask_graph_construction(args, scene_points, frame_list, dataset):
    with no_gc():
        return _mask_graph_construction(args, scene_points, frame_list, dataset)


def _mask_graph_construction(args, scene_points, frame_list, dataset):
    if args.debug:
        print('start building point in mask matrix')
    ctx, gi, gl, keys, mpc = _build(args, scene_points, frame_list, dataset)
    P, F, M = gi.num_points, gi.num_frames, gi.num_masks
    pfm_bits = ctx.point_frame_bits(P, F)
    pfm = PointFrameMatrix.from_bits(pfm_bits, F)
    if gi.threshold_status == MC_ERR_EMPTY_OBSERVERS:
        raise IndexError("index -1 is out of bounds for axis 0 with size 0")  # np.percentile([]) (:89)
    thr, isint = ctx.thresholds()
    vf = bits_to_bool(ctx.visible_frame_bits(M, F), F)
    c_off, c_idx = ctx.contained(M, gi.num_contained)
    node0 = ctx.nodes0(gi.num_nodes0)
    token = next(_tokens)
    _current["token"] = token
    src = Level0Source(gl, keys, vf, c_off, c_idx, M, mpc)
    handle = GraphHandle(token, len(node0), F, M, P, src, node0)
    nodes = Node.level0_list(src, node0.tolist(), handle)
    handle.nodes = tuple(nodes)
    return nodes, _thresholds(thr, isint), mpc, pfm


def build_point_in_mask_matrix(args, scene_points, frame_list, dataset):
    """construction.py:22-64 -> (boundary_points, point_in_mask_matrix, mask_point_clouds,
    point_frame_matrix, global_frame_mask_list)."""
    ctx, gi, gl, keys, mpc = _build(args, scene_points, frame_list, dataset)
    P, F = gi.num_points, gi.num_frames
    boundary = set(np.nonzero(ctx.boundary(P))[0].tolist())
    pim = ctx.point_in_mask(P, F).copy()
    pfm = bits_to_bool(ctx.point_frame_bits(P, F), F)
    return boundary, pim, mpc, pfm, gl


def _set_masks_from_sets(ctx, frame_list, global_frame_mask_list, mask_point_clouds, num_points):
    col_of = {}
    for c, fid in enumerate(frame_list):
        col_of.setdefault(fid, c)
    cols, labs, lens, chunks = [], [], [], []
    for fid, mid in global_frame_mask_list:
        s = np.fromiter(mask_point_clouds[f"{fid}_{mid}"], dtype=np.int64)
        cols.append(col_of[fid])
        labs.append(int(mid))
        lens.append(len(s))
        chunks.append(s.astype(np.int32))
    off = np.zeros(len(lens) + 1, np.int64)
    np.cumsum(lens, out=off[1:])
    pts = np.concatenate(chunks) if chunks else np.zeros(0, np.int32)
    ctx.set_masks(num_points, len(frame_list), cols, labs, off, pts)


def process_masks(frame_list, global_frame_mask_list, point_in_mask_matrix, boundary_points, mask_point_clouds, args):
    """construction.py:137-170 -> (visible_frames [M,F], contained_masks [M,M] float tensors, undersegment ids).
    The point-in-mask matrix and boundary set are recomputed on the device from the same masks."""
    import torch
    ctx = _device.context()
    _current["token"] = None
    P = int(np.asarray(point_in_mask_matrix).shape[0])
    _set_masks_from_sets(ctx, frame_list, global_frame_mask_list, mask_point_clouds, P)
    ctx.build(args.mask_visible_threshold, args.contained_threshold, args.undersegment_filter_threshold)
    gi = ctx.graph_info()
    M, F = gi.num_masks, gi.num_frames
    vf = bits_to_bool(ctx.visible_frame_bits(M, F), F).astype(np.float32)
    off, idx = ctx.contained(M, gi.num_contained)
    cm = np.zeros((M, M), np.float32)
    cm[np.repeat(np.arange(M), np.diff(off)), idx] = 1.0
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    return (torch.from_numpy(vf).to(dev), torch.from_numpy(cm).to(dev),
            [int(u) for u in ctx.undersegment(gi.num_undersegment)])


def get_observer_num_thresholds(visible_frames):
    """construction.py:80-96 (observer counts histogrammed on the device)."""
    vf = _device.as_numpy(visible_frames) > 0
    ctx = _device.context()
    try:
        thr, isint = ctx.observer_thresholds(bool_to_bits(vf), vf.shape[1])
    except McError as e:
        if e.code == MC_ERR_EMPTY_OBSERVERS:
            raise IndexError("index -1 is out of bounds for axis 0 with size 0") from e
        raise
    return _thresholds(thr, isint)


def init_nodes(global_frame_mask_list, mask_project_on_all_frames, contained_masks, undersegment_mask_ids,
               mask_point_clouds):
    """construction.py:66-78."""
    useg = set(int(u) for u in undersegment_mask_ids)
    vf = _device.as_numpy(mask_project_on_all_frames) > 0
    cm = _device.as_numpy(contained_masks) > 0
    nodes = []
    for g, (frame_id, mask_id) in enumerate(global_frame_mask_list):
        if g in useg:
            continue
        nodes.append(Node.compact([(frame_id, mask_id)], vf[g], np.nonzero(cm[g])[0], cm.shape[1],
                                  mask_point_clouds[f'{frame_id}_{mask_id}'], (0, len(nodes)), None))
    return nodes
