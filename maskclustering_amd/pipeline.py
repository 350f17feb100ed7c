"""G-variant runner: per-frame mask sets in → graph (S2–S5) → clustering (S6),
all on the device through libmcgraph.  Used by bench.py, __graft_entry__ and
the reference-API shims (maskclustering_amd/graph/*.py).

``canonical()`` exports every stage in the order-free form of the golden
fixtures (tests/golden/make_golden.py), so a run can be compared with the
reference's own outputs and with the CPU oracle bit for bit.
"""
from __future__ import annotations

import numpy as np

from . import _native


class GraphRun:
    """One scene on one device context."""

    def __init__(self, device: int = 0, ctx: _native.Context | None = None):
        self.ctx = ctx or _native.Context(device)
        self.P = self.F = 0

    # ---- inputs ---------------------------------------------------------------------
    def set_masks(self, num_points, num_frames, mask_col, mask_label, mask_off, mask_pts=None,
                  pts_device_ptr=None):
        self.P, self.F = int(num_points), int(num_frames)
        self.mask_col = np.asarray(mask_col, np.int32)
        self.mask_label = np.asarray(mask_label, np.int32)
        self.ctx.set_masks(num_points, num_frames, mask_col, mask_label, mask_off, mask_pts, pts_device_ptr)

    def set_scene(self, scene):
        self.set_masks(scene.num_points, scene.num_frames, scene.mask_col, scene.mask_label, scene.mask_off,
                       scene.mask_pts)

    # ---- device work (asynchronous on the context stream) -----------------------------
    def build(self, mask_visible_threshold, contained_threshold, undersegment_filter_threshold):
        self.ctx.build(mask_visible_threshold, contained_threshold, undersegment_filter_threshold)

    def cluster(self, connect_threshold, thresholds=None):
        """thresholds=None uses the device-computed ladder (construction.py:80-96)."""
        self.ctx.cluster(thresholds, connect_threshold)

    def step(self, mask_visible_threshold, undersegment_filter_threshold, view_consensus_threshold,
             contained_threshold):
        """One full pass of the hot path (S2–S6 + final point sets)."""
        self.build(mask_visible_threshold, contained_threshold, undersegment_filter_threshold)
        self.cluster(view_consensus_threshold)

    # ---- results --------------------------------------------------------------------
    def canonical(self, dense: bool = True) -> dict:
        """dense=False skips the point-in-mask and point-frame matrices (P×F: 3 GB / 0.2 GB at
        C3), for the large-scene parity tests."""
        c = self.ctx
        gi = c.graph_info()
        P, F, M = gi.num_points, gi.num_frames, gi.num_masks
        out = {}
        gidx = c.global_masks(M)
        out["_input_index"] = gidx
        out["gl_col"], out["gl_label"] = self.mask_col[gidx], self.mask_label[gidx]
        bnd = c.boundary(P)
        out["boundary"] = np.nonzero(bnd)[0].astype(np.int32)
        if dense:
            pim = c.point_in_mask(P, F)
            nzp, nzc = np.nonzero(pim)
            out["pim_p"], out["pim_c"], out["pim_v"] = nzp.astype(np.int32), nzc.astype(np.int32), \
                pim[nzp, nzc].astype(np.int32)
            out["pfm_bits"] = np.packbits(bits_to_bool(c.point_frame_bits(P, F), F), axis=1)
        out["vf_bits"] = np.packbits(bits_to_bool(c.visible_frame_bits(M, F), F), axis=1)
        off, idx = c.contained(M, gi.num_contained)
        rows = np.repeat(np.arange(M, dtype=np.int32), np.diff(off))
        out["c_row"], out["c_col"] = rows, idx.astype(np.int32)
        out["undersegment"] = c.undersegment(gi.num_undersegment)
        out["node0_g"] = c.nodes0(gi.num_nodes0)
        out["observer_hist"] = c.observer_hist(F)
        if gi.threshold_status == _native.MC_OK:
            thr, isint = c.thresholds()
        else:
            thr, isint = np.zeros(0, np.float32), np.zeros(0, bool)
        out["thr_value"], out["thr_is_int"] = thr, isint
        out.update(self.canonical_cluster(F, node0=out["node0_g"]))
        return out

    def canonical_cluster(self, F, node0=None) -> dict:
        """S6 results; ``node0`` maps level-0 node ids to global mask ids."""
        c = self.ctx
        ci = c.cluster_info()
        T = ci.num_iterations
        out = {"num_iters": np.array(T, np.int32)}
        sizes = c.level_sizes(T)
        out["level_sizes"] = sizes
        for t in range(T):
            out[f"part_{t}"] = c.partition(t, int(sizes[t]))
        out["edge_counts"] = c.edge_counts(T)
        obj = c.objects(ci, F)
        K = ci.num_objects
        out["obj_mask_off"] = obj["mask_off"]
        out["obj_mask_idx"] = obj["mask_idx"]  # level-0 node ids; callers map to masks
        out["obj_pt_off"], out["obj_pt_idx"] = obj["pt_off"], obj["pt_idx"]
        out["obj_vf_bits"] = np.packbits(bits_to_bool(obj["vf_bits"], F), axis=1) if K else np.zeros((0, (F + 7) // 8), np.uint8)
        out["obj_c_off"], out["obj_c_idx"] = obj["c_off"], obj["c_idx"]
        out["obj_node_info"] = np.array([(T, k) if T else (0, k) for k in range(K)], np.int32).reshape(-1, 2)
        if T:
            last = out[f"part_{T - 1}"]
            order = np.argsort(last, kind="stable")
            so = np.zeros(K + 1, np.int64)
            so[1:] = np.cumsum(np.bincount(last, minlength=K))
            out["obj_son_off"], out["obj_son_idx"] = so, order.astype(np.int32)
        else:
            out["obj_son_off"], out["obj_son_idx"] = np.zeros(K + 1, np.int64), np.zeros(0, np.int32)
        if node0 is not None:
            out["obj_mask_idx"] = node0[obj["mask_idx"]].astype(np.int32)
        return out


def bits_to_bool(words: np.ndarray, n: int) -> np.ndarray:
    """(R, W) uint64 little-endian bit rows -> (R, n) bool."""
    words = np.ascontiguousarray(words, dtype="<u8")
    if words.size == 0:
        return np.zeros((words.shape[0], n), bool)
    b = np.unpackbits(words.view(np.uint8).reshape(words.shape[0], -1), axis=1, bitorder="little")
    return b[:, :n].astype(bool)


def bool_to_bits(m: np.ndarray) -> np.ndarray:
    """(R, n) bool -> (R, ceil(n/64)) uint64 little-endian bit rows."""
    m = np.asarray(m, bool)
    R, n = m.shape
    W = (n + 63) // 64
    pad = np.zeros((R, W * 64), bool)
    pad[:, :n] = m
    return np.packbits(pad, axis=1, bitorder="little").view("<u8").reshape(R, W).copy()
