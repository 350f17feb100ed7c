"""ctypes binding of libmcgraph.so (the C-ABI in include/mcgraph.h).

The library is built in-tree by ``__graft_entry__.build()`` (hipcc, gfx950).
There is no fallback: if the shared object is missing or fails to load, every
entry point raises, so a GPU run can never silently take another path.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MCGRAPH_LIB") or os.path.join(HERE, "libmcgraph.so")  # override: profiling variants

MC_OK = 0
MC_ERR_INVALID = 1
MC_ERR_HIP = 2
MC_ERR_STATE = 3
MC_ERR_EMPTY_OBSERVERS = 4
MC_ERR_UNSUPPORTED = 5
MC_ERR_NO_NODES = 6

EXPORTED = [
    "mc_ctx_create", "mc_ctx_destroy", "mc_ctx_set_stream", "mc_ctx_get_stream", "mc_ctx_synchronize",
    "mc_ctx_last_error", "mc_ctx_set_timing", "mc_ctx_set_timing_filter", "mc_ctx_get_kernel_time", "mc_ctx_reset_kernel_times",
    "mc_debug_counters", "mc_ctx_set_memory_budget", "mc_scene_set_masks", "mc_graph_build", "mc_graph_get_info", "mc_graph_get_global_masks",
    "mc_graph_get_boundary", "mc_graph_get_point_in_mask", "mc_graph_get_point_frame_bits",
    "mc_graph_get_visible_frame_bits", "mc_graph_get_contained", "mc_graph_get_undersegment",
    "mc_graph_get_nodes0", "mc_graph_get_observer_hist", "mc_graph_get_thresholds", "mc_observer_thresholds",
    "mc_nodes_set",
    "mc_cluster_run", "mc_cluster_get_info", "mc_cluster_get_level_sizes", "mc_cluster_get_level_caps", "mc_cluster_get_partition",
    "mc_cluster_get_edge_counts", "mc_cluster_get_final_labels", "mc_cluster_get_objects",
    "mc_bp_params_default", "mc_scene_set_points", "mc_backproject", "mc_backproject_frames", "mc_backproject_frames_raw",
    "mc_backproject_get_info", "mc_backproject_get_batching",
    "mc_backproject_get_masks", "mc_backproject_get_candidates", "mc_scene_use_backprojection",
    "mc_backproject_copy_points_device",
    "mc_pp_run", "mc_pp_get_info", "mc_pp_get_results", "mc_eval_match_counts", "mc_frames_decode",
    "mc_shard_set", "mc_shard_pending", "mc_shard_export", "mc_shard_import",
    "mc_cluster_set_edge_capture", "mc_cluster_get_edges", "mc_openvoc_query", "mc_bits_unpack", "mc_setorder_replay",
    "mc_setorder_begin", "mc_setorder_finish", "mc_setorder_free",
    "mc_comm_unique_id", "mc_ctx_comm_init", "mc_ctx_attach_comm",
]
MC_COMM_ID_BYTES = 128

MC_SHARD_S3 = 1
MC_SHARD_HIST = 2
MC_SHARD_FOREST = 3

MC_BP_NSTAT = 10
BP_STATS = ["frame", "id", "npix", "nvox", "ndbscan", "nsor", "ncand", "ncovered", "nneighbors", "kept"]


class McError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"libmcgraph error {code}: {msg}")
        self.code = code


class GraphParams(ctypes.Structure):
    _fields_ = [("mask_visible_threshold", ctypes.c_double),
                ("contained_threshold", ctypes.c_double),
                ("undersegment_filter_threshold", ctypes.c_double)]


class GraphInfo(ctypes.Structure):
    _fields_ = [("num_points", ctypes.c_int64), ("num_frames", ctypes.c_int32), ("num_masks", ctypes.c_int32),
                ("num_undersegment", ctypes.c_int32), ("num_nodes0", ctypes.c_int32),
                ("num_contained", ctypes.c_int64), ("num_boundary", ctypes.c_int64),
                ("num_thresholds", ctypes.c_int32), ("threshold_status", ctypes.c_int32)]


class ClusterInfo(ctypes.Structure):
    _fields_ = [("num_iterations", ctypes.c_int32), ("num_objects", ctypes.c_int32),
                ("num_nodes0", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("num_object_points", ctypes.c_int64), ("num_object_contained", ctypes.c_int64),
                ("num_object_masks", ctypes.c_int64)]


class BpParams(ctypes.Structure):
    """mc_bp_params: the S1 constants (utils/mask_backprojection.py:8-14,38; utils/geometry.py:10,16,22)."""
    _fields_ = [("depth_trunc", ctypes.c_double), ("voxel_size", ctypes.c_double),
                ("dbscan_eps", ctypes.c_double), ("component_min_fraction", ctypes.c_double),
                ("sor_std_ratio", ctypes.c_double), ("ball_radius", ctypes.c_double),
                ("coverage_threshold", ctypes.c_double), ("dbscan_min_points", ctypes.c_int32),
                ("sor_neighbors", ctypes.c_int32), ("ball_k", ctypes.c_int32), ("few_points", ctypes.c_int32)]


class BpInfo(ctypes.Structure):
    _fields_ = [("num_frames", ctypes.c_int32), ("num_candidates", ctypes.c_int32), ("num_masks", ctypes.c_int32),
                ("error_frame", ctypes.c_int32), ("num_mask_points", ctypes.c_int64)]


class PPParams(ctypes.Structure):
    """mc_pp_params: utils/post_process.py:104,109 (DBSCAN), :95 (point filter), :194 (overlap)."""
    _fields_ = [("dbscan_eps", ctypes.c_double), ("dbscan_min_points", ctypes.c_int32),
                ("point_filter_threshold", ctypes.c_double), ("overlapping_ratio", ctypes.c_double)]


class PPInfo(ctypes.Structure):
    _fields_ = [("num_objects", ctypes.c_int32), ("num_filtered", ctypes.c_int32), ("num_final", ctypes.c_int32),
                ("num_entries", ctypes.c_int64), ("num_node_masks", ctypes.c_int64)]


_lib = None


def load():
    """Load libmcgraph.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: run __graft_entry__.build() (hipcc --offload-arch=gfx950)")
    # One HIP runtime per process: torch bundles its own libamdhip64.so.7 (same soname as
    # /opt/rocm's).  Whichever is loaded first serves both, and torch cannot initialise the GPU
    # on a runtime it was not built with, so torch's is loaded before this library when present.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, i64, dbl = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_double
    P = ctypes.POINTER
    sig = {
        "mc_ctx_create": (ctypes.c_int, [ctypes.c_int, P(vp)]),
        "mc_ctx_destroy": (None, [vp]),
        "mc_ctx_set_stream": (ctypes.c_int, [vp, vp]),
        "mc_ctx_get_stream": (vp, [vp]),
        "mc_ctx_synchronize": (ctypes.c_int, [vp]),
        "mc_ctx_last_error": (ctypes.c_char_p, [vp]),
        "mc_ctx_set_timing": (ctypes.c_int, [vp, ctypes.c_int]),
        "mc_ctx_set_timing_filter": (ctypes.c_int, [vp, ctypes.c_char_p]),
        "mc_ctx_get_kernel_time": (ctypes.c_int, [vp, ctypes.c_char_p, P(dbl), P(i64)]),
        "mc_ctx_reset_kernel_times": (ctypes.c_int, [vp]),
        "mc_debug_counters": (ctypes.c_int, [vp, vp, i32, ctypes.c_int]),
        "mc_ctx_set_memory_budget": (ctypes.c_int, [vp, i64]),
        "mc_scene_set_masks": (ctypes.c_int, [vp, i64, i32, i32, vp, vp, vp, vp, ctypes.c_int]),
        "mc_graph_build": (ctypes.c_int, [vp, P(GraphParams)]),
        "mc_graph_get_info": (ctypes.c_int, [vp, P(GraphInfo)]),
        "mc_graph_get_global_masks": (ctypes.c_int, [vp, vp]),
        "mc_graph_get_boundary": (ctypes.c_int, [vp, vp]),
        "mc_graph_get_point_in_mask": (ctypes.c_int, [vp, vp]),
        "mc_graph_get_point_frame_bits": (ctypes.c_int, [vp, vp]),
        "mc_graph_get_visible_frame_bits": (ctypes.c_int, [vp, vp]),
        "mc_graph_get_contained": (ctypes.c_int, [vp, vp, vp]),
        "mc_graph_get_undersegment": (ctypes.c_int, [vp, vp]),
        "mc_graph_get_nodes0": (ctypes.c_int, [vp, vp]),
        "mc_graph_get_observer_hist": (ctypes.c_int, [vp, vp]),
        "mc_graph_get_thresholds": (ctypes.c_int, [vp, vp, vp, P(i32)]),
        "mc_observer_thresholds": (ctypes.c_int, [vp, i32, i32, vp, vp, vp, P(i32)]),
        "mc_nodes_set": (ctypes.c_int, [vp, i32, i32, i32, i64, vp, vp, vp, vp, vp]),
        "mc_cluster_run": (ctypes.c_int, [vp, vp, i32, dbl]),
        "mc_cluster_get_info": (ctypes.c_int, [vp, P(ClusterInfo)]),
        "mc_cluster_get_level_sizes": (ctypes.c_int, [vp, vp]),
        "mc_cluster_get_level_caps": (ctypes.c_int, [vp, vp]),
        "mc_cluster_get_partition": (ctypes.c_int, [vp, i32, vp]),
        "mc_cluster_get_edge_counts": (ctypes.c_int, [vp, vp]),
        "mc_cluster_get_final_labels": (ctypes.c_int, [vp, vp]),
        "mc_cluster_get_objects": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, vp]),
        "mc_bp_params_default": (None, [P(BpParams)]),
        "mc_scene_set_points": (ctypes.c_int, [vp, i64, vp, ctypes.c_int]),
        "mc_backproject": (ctypes.c_int, [vp, i32, i32, i32, vp, vp, vp, vp, ctypes.c_int, P(BpParams)]),
        "mc_backproject_frames": (ctypes.c_int, [vp, i32, i32, i32, vp, vp, vp, vp, P(BpParams)]),
        "mc_backproject_frames_raw": (ctypes.c_int, [vp, i32, i32, i32, vp, ctypes.c_double, vp, vp, vp, P(BpParams)]),
        "mc_backproject_get_info": (ctypes.c_int, [vp, P(BpInfo)]),
        "mc_backproject_get_batching": (ctypes.c_int, [vp, vp]),
        "mc_backproject_get_masks": (ctypes.c_int, [vp, vp, vp, vp, vp]),
        "mc_backproject_copy_points_device": (ctypes.c_int, [vp, vp]),
        "mc_backproject_get_candidates": (ctypes.c_int, [vp, vp]),
        "mc_scene_use_backprojection": (ctypes.c_int, [vp]),
        "mc_pp_run": (ctypes.c_int, [vp, P(PPParams), i64, i32, vp, vp, i32, vp, vp, i32, vp, vp, vp, vp, vp, vp]),
        "mc_pp_get_info": (ctypes.c_int, [vp, P(PPInfo)]),
        "mc_pp_get_results": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp]),
        "mc_eval_match_counts": (ctypes.c_int, [vp, i64, i32, vp, vp, i32, vp, vp, vp, vp]),
        "mc_frames_decode": (ctypes.c_int, [vp, i32, i32, i32, vp, dbl, i32, i32, vp, ctypes.c_int, vp, vp]),
        "mc_shard_set": (ctypes.c_int, [vp, i32, i32]),
        "mc_cluster_set_edge_capture": (ctypes.c_int, [vp, i64]),
        "mc_openvoc_query": (ctypes.c_int, [vp, i32, vp, vp, i32, i32, vp, i32, vp, ctypes.c_float, vp]),
        "mc_bits_unpack": (ctypes.c_int, [vp, ctypes.c_int64, i32, i32, vp]),
        "mc_setorder_replay": (ctypes.c_int, [i32, vp, vp, vp, vp, vp, vp, i32, P(i32), vp, vp, vp, vp, vp, vp, vp]),
        "mc_setorder_begin": (ctypes.c_int, [i32, vp, vp, vp, i32, ctypes.c_int, P(vp)]),
        "mc_setorder_finish": (ctypes.c_int, [vp, i32, vp, vp, vp, vp, P(i32), vp, vp, vp, vp, vp, vp, vp]),
        "mc_setorder_free": (None, [vp]),
        "mc_cluster_get_edges": (ctypes.c_int, [vp, vp, P(i64)]),
        "mc_shard_pending": (ctypes.c_int, [vp, P(i32)]),
        "mc_shard_export": (ctypes.c_int, [vp, i32, vp, P(i64)]),
        "mc_shard_import": (ctypes.c_int, [vp, i32, vp, i64]),
        "mc_comm_unique_id": (ctypes.c_int, [vp]),
        "mc_ctx_comm_init": (ctypes.c_int, [vp, vp, i32, i32]),
        "mc_ctx_attach_comm": (ctypes.c_int, [vp, vp]),
    }
    # MCGRAPH_LIB_PARTIAL=1 (A/B scripts only): an older variant library may lack newer entry points
    partial = os.environ.get("MCGRAPH_LIB_PARTIAL") == "1"
    for name, (res, args) in sig.items():
        if partial and not hasattr(L, name):
            continue
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def comm_unique_id() -> bytes:
    """mc_comm_unique_id (ncclGetUniqueId): made on one rank, broadcast to the others."""
    buf = ctypes.create_string_buffer(MC_COMM_ID_BYTES)
    rc = load().mc_comm_unique_id(buf)
    if rc != MC_OK:
        raise McError(rc, "mc_comm_unique_id failed (RCCL not loadable?)")
    return buf.raw


def _ptr(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


def setorder_replay(level_sizes, edge_off, edge_a, edge_b, pt_off, pts, threads=0, labels=False):
    """mc_setorder_replay (host only, no device): the reference's container orders of a clustering run
    (include/mcgraph.h).  Returns dict(mask_off, mask_order, pt_off, pts, son_off, son_order[, labels])."""
    L = load()
    T = len(level_sizes)
    sz = np.ascontiguousarray(level_sizes, np.int32)
    eo = np.ascontiguousarray(edge_off, np.int64)
    ea = np.ascontiguousarray(edge_a, np.int32)
    eb = np.ascontiguousarray(edge_b, np.int32)
    po = np.ascontiguousarray(pt_off, np.int64)
    pp = np.ascontiguousarray(pts, np.int32)
    N0, NL = int(sz[0]), int(sz[T - 1])
    K = ctypes.c_int32()
    mo, mord = np.zeros(NL + 1, np.int64), np.zeros(max(N0, 1), np.int32)
    oo, opts = np.zeros(NL + 1, np.int64), np.zeros(max(int(po[N0]), 1), np.int32)
    so, sord = np.zeros(NL + 1, np.int64), np.zeros(max(NL, 1), np.int32)
    lab = np.zeros(max(int(sz.sum()), 1), np.int32) if labels else None
    rc = L.mc_setorder_replay(T, _ptr(sz), _ptr(eo), _ptr(ea), _ptr(eb), _ptr(po), _ptr(pp), int(threads),
                              ctypes.byref(K), _ptr(mo), _ptr(mord), _ptr(oo), _ptr(opts), _ptr(so), _ptr(sord),
                              _ptr(lab))
    if rc != MC_OK:
        raise McError(rc, "mc_setorder_replay: inconsistent levels / edges / point sets")
    k = K.value
    out = dict(mask_off=mo[:k + 1], mask_order=mord[:N0], pt_off=oo[:k + 1], pts=opts[:int(oo[k])],
               son_off=so[:k + 1], son_order=sord[:NL])
    if labels:
        out["labels"] = lab[:int(sz.sum())]
    return out


class SetOrder:
    """mc_setorder_begin / mc_setorder_finish: the level-0 point sets (node i: pts[node_start[i] :
    node_start[i] + node_len[i]], added in order) built on a native background thread from
    construction on, the iterations replayed by finish (the result of setorder_replay)."""

    def __init__(self, node_start, node_len, pts, threads=0, async_build=True):
        self.L = load()
        st = np.ascontiguousarray(node_start, np.int64)
        ln = np.ascontiguousarray(node_len, np.int64)
        pp = np.ascontiguousarray(pts, np.int32)
        if len(st) != len(ln) or (len(ln) and int((st + ln).max()) > len(pp)):
            raise ValueError("node ranges outside pts")
        self._keep = (st, ln, pp)  # read by the background thread until finish / close
        self.n0, self.total = len(st), int(ln.sum())
        h = ctypes.c_void_p()
        rc = self.L.mc_setorder_begin(self.n0, _ptr(st), _ptr(ln), _ptr(pp), int(threads), 1 if async_build else 0,
                                      ctypes.byref(h))
        if rc != MC_OK:
            raise McError(rc, "mc_setorder_begin: invalid node ranges / point ids")
        self.h = h

    def finish(self, level_sizes, edge_off, edge_a, edge_b, labels=False):
        if not getattr(self, "h", None):
            raise RuntimeError("SetOrder already finished")
        T = len(level_sizes)
        sz = np.ascontiguousarray(level_sizes, np.int32)
        eo = np.ascontiguousarray(edge_off, np.int64)
        ea = np.ascontiguousarray(edge_a, np.int32)
        eb = np.ascontiguousarray(edge_b, np.int32)
        N0, NL = int(sz[0]), int(sz[T - 1])
        K = ctypes.c_int32()
        mo, mord = np.zeros(NL + 1, np.int64), np.zeros(max(N0, 1), np.int32)
        oo, opts = np.zeros(NL + 1, np.int64), np.zeros(max(self.total, 1), np.int32)
        so, sord = np.zeros(NL + 1, np.int64), np.zeros(max(NL, 1), np.int32)
        lab = np.zeros(max(int(sz.sum()), 1), np.int32) if labels else None
        try:
            rc = self.L.mc_setorder_finish(self.h, T, _ptr(sz), _ptr(eo), _ptr(ea), _ptr(eb), ctypes.byref(K), _ptr(mo),
                                           _ptr(mord), _ptr(oo), _ptr(opts), _ptr(so), _ptr(sord), _ptr(lab))
        finally:
            self.close()
        if rc != MC_OK:
            raise McError(rc, "mc_setorder_finish: inconsistent levels / edges, or a negative point id")
        k = K.value
        out = dict(mask_off=mo[:k + 1], mask_order=mord[:N0], pt_off=oo[:k + 1], pts=opts[:int(oo[k])],
                   son_off=so[:k + 1], son_order=sord[:NL])
        if labels:
            out["labels"] = lab[:int(sz.sum())]
        return out

    def close(self):
        if getattr(self, "h", None):
            self.L.mc_setorder_free(self.h)
            self.h = None
        self._keep = None

    def __del__(self):
        self.close()


class Context:
    """One libmcgraph context (device memory + stream) — one scene at a time."""

    def __init__(self, device: int = 0):
        self.device_index = int(device)
        self.L = load()
        h = ctypes.c_void_p()
        rc = self.L.mc_ctx_create(int(device), ctypes.byref(h))
        if rc != MC_OK:
            raise McError(rc, "mc_ctx_create failed (no HIP device?)")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self.L.mc_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != MC_OK:
            raise McError(rc, self.L.mc_ctx_last_error(self.h).decode())

    # ---- context ----
    def set_stream(self, stream_handle):
        self._check(self.L.mc_ctx_set_stream(self.h, ctypes.c_void_p(stream_handle) if stream_handle else None))

    def stream(self):
        return self.L.mc_ctx_get_stream(self.h)

    def synchronize(self):
        self._check(self.L.mc_ctx_synchronize(self.h))

    def set_timing(self, on: bool):
        self._check(self.L.mc_ctx_set_timing(self.h, 1 if on else 0))

    def set_timing_filter(self, name):
        self._check(self.L.mc_ctx_set_timing_filter(self.h, name.encode() if name else None))

    def kernel_time(self, name: str):
        ms, n = ctypes.c_double(), ctypes.c_int64()
        self._check(self.L.mc_ctx_get_kernel_time(self.h, name.encode(), ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def reset_kernel_times(self):
        self._check(self.L.mc_ctx_reset_kernel_times(self.h))

    def set_memory_budget(self, nbytes: int):
        """mc_ctx_set_memory_budget: HBM bytes S1's per-batch arrays may take (0 = the default share)."""
        self._check(self.L.mc_ctx_set_memory_budget(self.h, int(nbytes)))

    def debug_counters(self, reset: bool = False):
        """(checks compiled in, failures per check kind): the in-kernel invariant checks of a
        -DMC_DBG_CHECK=1 build (docs/experiments.md); a normal build reports (False, zeros)."""
        out = np.zeros(9, np.int64)
        self._check(self.L.mc_debug_counters(self.h, _ptr(out), 9, 1 if reset else 0))
        return bool(out[0]), out[1:]

    # ---- row-block sharding over processes (include/mcgraph.h) ----
    @property
    def torch_device(self):
        import torch
        return torch.device("cuda", self.device_index)

    def shard_set(self, rank, world):
        self._check(self.L.mc_shard_set(self.h, int(rank), int(world)))

    def comm_init(self, unique_id: bytes, rank: int, world: int):
        """mc_ctx_comm_init: an RCCL communicator owned by the context (rank / world of the sharded
        graph stages come from it; the exchanges then run inside mc_graph_build / mc_cluster_run)."""
        assert len(unique_id) == MC_COMM_ID_BYTES
        buf = ctypes.create_string_buffer(bytes(unique_id), MC_COMM_ID_BYTES)
        self._check(self.L.mc_ctx_comm_init(self.h, buf, int(rank), int(world)))

    def attach_comm(self, nccl_comm):
        """mc_ctx_attach_comm: a caller-owned ncclComm_t (an int address); None detaches."""
        self._check(self.L.mc_ctx_attach_comm(self.h, None if nccl_comm is None else ctypes.c_void_p(int(nccl_comm))))

    def shard_pending(self) -> int:
        ph = ctypes.c_int32()
        self._check(self.L.mc_shard_pending(self.h, ctypes.byref(ph)))
        return ph.value

    def shard_export_size(self, phase) -> int:
        n = ctypes.c_int64()
        self._check(self.L.mc_shard_export(self.h, int(phase), None, ctypes.byref(n)))
        return n.value

    def shard_export(self, phase, out):
        """this rank's block into the device tensor ``out`` (stream-ordered on the context stream)"""
        n = ctypes.c_int64()
        self._check(self.L.mc_shard_export(self.h, int(phase), ctypes.c_void_p(out.data_ptr()), ctypes.byref(n)))

    def shard_import(self, phase, blocks, stride_bytes):
        """every rank's block ([world][stride_bytes] in rank order; HIST: the summed block)"""
        self._check(self.L.mc_shard_import(self.h, int(phase), ctypes.c_void_p(blocks.data_ptr()), int(stride_bytes)))

    # ---- scene ----
    def set_masks(self, num_points, num_frames, mask_col, mask_label, mask_off, mask_pts=None, pts_device_ptr=None):
        col = np.ascontiguousarray(mask_col, np.int32)
        lab = np.ascontiguousarray(mask_label, np.int32)
        off = np.ascontiguousarray(mask_off, np.int64)
        if pts_device_ptr is not None:
            pts_p, on_dev = ctypes.c_void_p(int(pts_device_ptr)), 1
        else:
            pts = np.ascontiguousarray(mask_pts, np.int32)
            self._keep_pts = pts
            pts_p, on_dev = _ptr(pts), 0
        self._check(self.L.mc_scene_set_masks(self.h, int(num_points), int(num_frames), len(col), _ptr(col),
                                               _ptr(lab), _ptr(off), pts_p, on_dev))

    def build(self, mask_visible_threshold, contained_threshold, undersegment_filter_threshold):
        prm = GraphParams(float(mask_visible_threshold), float(contained_threshold),
                          float(undersegment_filter_threshold))
        self._check(self.L.mc_graph_build(self.h, ctypes.byref(prm)))

    def graph_info(self) -> GraphInfo:
        info = GraphInfo()
        self._check(self.L.mc_graph_get_info(self.h, ctypes.byref(info)))
        return info

    def global_masks(self, M):
        out = np.zeros(max(M, 1), np.int32)
        self._check(self.L.mc_graph_get_global_masks(self.h, _ptr(out)))
        return out[:M]

    def boundary(self, P):
        out = np.zeros(max(P, 1), np.uint8)
        self._check(self.L.mc_graph_get_boundary(self.h, _ptr(out)))
        return out[:P]

    def point_in_mask(self, P, F):
        out = np.zeros((max(P, 1), max(F, 1)), np.uint16)
        self._check(self.L.mc_graph_get_point_in_mask(self.h, _ptr(out)))
        return out[:P, :F]

    def point_frame_bits(self, P, F):
        FW = (F + 63) // 64
        out = np.zeros((max(P, 1), max(FW, 1)), np.uint64)
        self._check(self.L.mc_graph_get_point_frame_bits(self.h, _ptr(out)))
        return out[:P, :FW]

    def visible_frame_bits(self, M, F):
        FW = (F + 63) // 64
        out = np.zeros((max(M, 1), max(FW, 1)), np.uint64)
        self._check(self.L.mc_graph_get_visible_frame_bits(self.h, _ptr(out)))
        return out[:M, :FW]

    def contained(self, M, nnz):
        off = np.zeros(M + 1, np.int64)
        idx = np.zeros(max(nnz, 1), np.int32)
        self._check(self.L.mc_graph_get_contained(self.h, _ptr(off), _ptr(idx)))
        return off, idx[:nnz]

    def undersegment(self, n):
        out = np.zeros(max(n, 1), np.int32)
        self._check(self.L.mc_graph_get_undersegment(self.h, _ptr(out)))
        return out[:n]

    def nodes0(self, n):
        out = np.zeros(max(n, 1), np.int32)
        self._check(self.L.mc_graph_get_nodes0(self.h, _ptr(out)))
        return out[:n]

    def observer_hist(self, F):
        out = np.zeros(F + 1, np.uint64)
        self._check(self.L.mc_graph_get_observer_hist(self.h, _ptr(out)))
        return out

    def thresholds(self):
        thr = np.zeros(20, np.float32)
        isint = np.zeros(20, np.int32)
        n = ctypes.c_int32()
        self._check(self.L.mc_graph_get_thresholds(self.h, _ptr(thr), _ptr(isint), ctypes.byref(n)))
        return thr[:n.value].copy(), isint[:n.value].astype(bool)

    def observer_thresholds(self, vf_bits, num_frames):
        """get_observer_num_thresholds (construction.py:80-96) on explicit VF bit rows."""
        vf = np.ascontiguousarray(vf_bits, np.uint64)
        thr = np.zeros(20, np.float32)
        isint = np.zeros(20, np.int32)
        n = ctypes.c_int32()
        self._check(self.L.mc_observer_thresholds(self.h, vf.shape[0], int(num_frames), _ptr(vf), _ptr(thr),
                                                  _ptr(isint), ctypes.byref(n)))
        return thr[:n.value].copy(), isint[:n.value].astype(bool)

    # ---- nodes / clustering ----
    def set_nodes(self, num_frames, num_masks, num_points, vf_bits, c_off, c_idx, pt_off, pt_idx):
        vf = np.ascontiguousarray(vf_bits, np.uint64)
        c_off = np.ascontiguousarray(c_off, np.int64)
        c_idx = np.ascontiguousarray(c_idx, np.int32)
        pt_off = np.ascontiguousarray(pt_off, np.int64)
        pt_idx = np.ascontiguousarray(pt_idx, np.int32)
        n = len(c_off) - 1
        self._check(self.L.mc_nodes_set(self.h, n, int(num_frames), int(num_masks), int(num_points), _ptr(vf),
                                        _ptr(c_off), _ptr(c_idx), _ptr(pt_off), _ptr(pt_idx)))

    def cluster(self, thresholds, connect_threshold):
        if thresholds is None:
            self._check(self.L.mc_cluster_run(self.h, None, 0, float(connect_threshold)))
        else:
            thr = np.ascontiguousarray(np.asarray(thresholds, dtype=np.float32))
            self._check(self.L.mc_cluster_run(self.h, _ptr(thr), len(thr), float(connect_threshold)))

    def cluster_info(self) -> ClusterInfo:
        info = ClusterInfo()
        self._check(self.L.mc_cluster_get_info(self.h, ctypes.byref(info)))
        return info

    def level_sizes(self, n_iter):
        out = np.zeros(n_iter + 1, np.int32)
        self._check(self.L.mc_cluster_get_level_sizes(self.h, _ptr(out)))
        return out

    def set_edge_capture(self, capacity):
        self._check(self.L.mc_cluster_set_edge_capture(self.h, int(capacity)))

    def edges(self):
        """captured edges as (t, a, b) int64 arrays, sorted by (t, a, b)"""
        n = ctypes.c_int64()
        self._check(self.L.mc_cluster_get_edges(self.h, None, ctypes.byref(n)))
        keys = np.zeros(max(n.value, 1), np.uint64)
        self._check(self.L.mc_cluster_get_edges(self.h, _ptr(keys), ctypes.byref(n)))
        keys = np.sort(keys[:n.value])
        return ((keys >> np.uint64(48)).astype(np.int64), ((keys >> np.uint64(24)) & np.uint64(0xffffff)).astype(np.int64),
                (keys & np.uint64(0xffffff)).astype(np.int64))

    def level_caps(self, n_iter):
        out = np.zeros(n_iter + 1, np.int32)
        self._check(self.L.mc_cluster_get_level_caps(self.h, _ptr(out)))
        return out

    def partition(self, t, n):
        out = np.zeros(max(n, 1), np.int32)
        self._check(self.L.mc_cluster_get_partition(self.h, int(t), _ptr(out)))
        return out[:n]

    def edge_counts(self, n_iter):
        out = np.zeros(max(n_iter, 1), np.int64)
        self._check(self.L.mc_cluster_get_edge_counts(self.h, _ptr(out)))
        return out[:n_iter]

    def final_labels(self, n0):
        out = np.zeros(max(n0, 1), np.int32)
        self._check(self.L.mc_cluster_get_final_labels(self.h, _ptr(out)))
        return out[:n0]

    def objects(self, info: ClusterInfo, F):
        K = info.num_objects
        FW = (F + 63) // 64
        vf = np.zeros((max(K, 1), max(FW, 1)), np.uint64)
        c_off = np.zeros(K + 1, np.int64)
        c_idx = np.zeros(max(info.num_object_contained, 1), np.int32)
        pt_off = np.zeros(K + 1, np.int64)
        pt_idx = np.zeros(max(info.num_object_points, 1), np.int32)
        m_off = np.zeros(K + 1, np.int64)
        m_idx = np.zeros(max(info.num_object_masks, 1), np.int32)
        self._check(self.L.mc_cluster_get_objects(self.h, _ptr(vf), _ptr(c_off), _ptr(c_idx), _ptr(pt_off),
                                                  _ptr(pt_idx), _ptr(m_off), _ptr(m_idx)))
        return dict(vf_bits=vf[:K, :FW], c_off=c_off, c_idx=c_idx[:c_off[-1]], pt_off=pt_off,
                    pt_idx=pt_idx[:pt_off[-1]], mask_off=m_off, mask_idx=m_idx[:m_off[-1]])


def bp_params(**kw) -> BpParams:
    """The reference's S1 constants, with optional overrides."""
    p = BpParams()
    load().mc_bp_params_default(ctypes.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def _bp_methods():
    def set_points(self, xyz=None, device_ptr=None, num_points=None):
        """Scene points as float32 [P,3] (construction.py:37 casts them to float32)."""
        if device_ptr is not None:
            self._check(self.L.mc_scene_set_points(self.h, int(num_points), ctypes.c_void_p(int(device_ptr)), 1))
            return
        pts = np.ascontiguousarray(xyz, np.float32).reshape(-1, 3)
        self._check(self.L.mc_scene_set_points(self.h, len(pts), _ptr(pts), 0))

    def backproject(self, depth, seg, intrinsics, poses, params: BpParams | None = None, device_ptrs=None,
                    shape=None):
        """S1 for a batch of frames: depth float32 [F,H,W], seg uint8 [F,H,W], intrinsics [F,4],
        poses [F,4,4].  device_ptrs = (depth, seg, intrinsics, poses) device pointers with shape=(F,H,W)."""
        prm = params or bp_params()
        if device_ptrs is not None:
            F, H, W = shape
            d, s_, k, t = (ctypes.c_void_p(int(x)) for x in device_ptrs)
            self._check(self.L.mc_backproject(self.h, F, H, W, d, s_, k, t, 1, ctypes.byref(prm)))
            return
        depth = np.ascontiguousarray(depth, np.float32)
        seg = np.ascontiguousarray(seg, np.uint8)
        F, H, W = depth.shape
        assert seg.shape == depth.shape
        K = np.ascontiguousarray(intrinsics, np.float64).reshape(F, 4)
        T = np.ascontiguousarray(poses, np.float64).reshape(F, 16)
        self._check(self.L.mc_backproject(self.h, F, H, W, _ptr(depth), _ptr(seg), _ptr(K), _ptr(T), 0,
                                          ctypes.byref(prm)))

    def backproject_frames(self, depth_frames, seg_frames, intrinsics, poses, params: BpParams | None = None,
                           depth_scale=None):
        """S1 from per-frame host arrays (depth float32 [H,W], seg uint8 [H,W] each, C-contiguous),
        staged to the device without an [F,H,W] host copy (mc_backproject_frames).  With
        depth_scale, the depth frames are the PNGs' uint16 values, decoded on the device
        (mc_backproject_frames_raw)."""
        prm = params or bp_params()
        F = len(depth_frames)
        assert len(seg_frames) == F and F > 0
        H, W = depth_frames[0].shape
        dt = np.float32 if depth_scale is None else np.uint16
        for d, sg in zip(depth_frames, seg_frames):
            if d.shape != (H, W) or sg.shape != (H, W) or d.dtype != dt or sg.dtype != np.uint8 \
                    or not d.flags.c_contiguous or not sg.flags.c_contiguous:
                raise ValueError(f"frames must be C-contiguous {np.dtype(dt).name} depth / uint8 seg arrays of one shape")
        dp = (ctypes.c_void_p * F)(*[d.ctypes.data for d in depth_frames])
        sp = (ctypes.c_void_p * F)(*[sg.ctypes.data for sg in seg_frames])
        K = np.ascontiguousarray(intrinsics, np.float64).reshape(F, 4)
        T = np.ascontiguousarray(poses, np.float64).reshape(F, 16)
        if depth_scale is None:
            self._check(self.L.mc_backproject_frames(self.h, F, H, W, dp, sp, _ptr(K), _ptr(T), ctypes.byref(prm)))
        else:
            self._check(self.L.mc_backproject_frames_raw(self.h, F, H, W, dp, float(depth_scale), sp, _ptr(K), _ptr(T),
                                                         ctypes.byref(prm)))

    def bp_info(self) -> BpInfo:
        info = BpInfo()
        self._check(self.L.mc_backproject_get_info(self.h, ctypes.byref(info)))
        return info

    def bp_batching(self) -> dict:
        """mc_backproject_get_batching: S1's frames per batch (last call), mask-pixel capacity, the
        bytes the per-batch arrays hold, and the batches redone after a mask-pixel overflow."""
        out = np.zeros(4, np.int64)
        self._check(self.L.mc_backproject_get_batching(self.h, _ptr(out)))
        return dict(frames_per_batch=int(out[0]), mask_pixel_cap=int(out[1]), bytes_held=int(out[2]),
                    redone=int(out[3]))

    def bp_masks(self):
        info = self.bp_info()
        M = info.num_masks
        col = np.zeros(max(M, 1), np.int32)
        lab = np.zeros(max(M, 1), np.int32)
        off = np.zeros(M + 1, np.int64)
        pts = np.zeros(max(info.num_mask_points, 1), np.int32)
        self._check(self.L.mc_backproject_get_masks(self.h, _ptr(col), _ptr(lab), _ptr(off), _ptr(pts)))
        return col[:M], lab[:M], off, pts[:info.num_mask_points]

    def bp_mask_index(self):
        """(mask_col, mask_label, mask_off) of the back-projected masks, without the point lists."""
        M = self.bp_info().num_masks
        col = np.zeros(max(M, 1), np.int32)
        lab = np.zeros(max(M, 1), np.int32)
        off = np.zeros(M + 1, np.int64)
        self._check(self.L.mc_backproject_get_masks(self.h, _ptr(col), _ptr(lab), _ptr(off), None))
        return col[:M], lab[:M], off

    def bp_points_to_device(self, dst_ptr):
        """Stream-ordered device-to-device copy of the mask point lists (int32) to dst_ptr."""
        self._check(self.L.mc_backproject_copy_points_device(self.h, ctypes.c_void_p(int(dst_ptr))))

    def bp_candidates(self):
        n = self.bp_info().num_candidates
        st = np.zeros((max(n, 1), MC_BP_NSTAT), np.int32)
        self._check(self.L.mc_backproject_get_candidates(self.h, _ptr(st)))
        return st[:n]

    def use_backprojection(self):
        self._check(self.L.mc_scene_use_backprojection(self.h))

    for f in (set_points, backproject, backproject_frames, bp_info, bp_batching, bp_masks, bp_mask_index,
              bp_points_to_device, bp_candidates, use_backprojection):
        setattr(Context, f.__name__, f)


_bp_methods()


def _pp_methods():
    def pp_run(self, params: PPParams, scene_xyz, pfm_bits, num_frames, mask_off, mask_pts, node_vf_bits,
               node_pt_off, node_pts, node_mask_off, node_masks, node_mask_col):
        a = dict(scene=np.ascontiguousarray(scene_xyz, np.float64), pfm=np.ascontiguousarray(pfm_bits, np.uint64),
                 moff=np.ascontiguousarray(mask_off, np.int64), mpts=np.ascontiguousarray(mask_pts, np.int32),
                 vf=np.ascontiguousarray(node_vf_bits, np.uint64), poff=np.ascontiguousarray(node_pt_off, np.int64),
                 pts=np.ascontiguousarray(node_pts, np.int32), qoff=np.ascontiguousarray(node_mask_off, np.int64),
                 qm=np.ascontiguousarray(node_masks, np.int32), qc=np.ascontiguousarray(node_mask_col, np.int32))
        self._check(self.L.mc_pp_run(self.h, ctypes.byref(params), a["scene"].shape[0], int(num_frames), _ptr(a["scene"]),
                                     _ptr(a["pfm"]), len(a["moff"]) - 1, _ptr(a["moff"]), _ptr(a["mpts"]),
                                     len(a["poff"]) - 1, _ptr(a["vf"]), _ptr(a["poff"]), _ptr(a["pts"]), _ptr(a["qoff"]),
                                     _ptr(a["qm"]), _ptr(a["qc"])))

    def pp_info(self) -> PPInfo:
        info = PPInfo()
        self._check(self.L.mc_pp_get_info(self.h, ctypes.byref(info)))
        return info

    def pp_results(self):
        i = self.pp_info()
        K, E, Q = i.num_objects, i.num_entries, i.num_node_masks
        r = dict(entry_object=np.zeros(max(E, 1), np.int32), mask_object=np.zeros(max(Q, 1), np.int32),
                 mask_coverage=np.zeros(max(Q, 1), np.float64), object_state=np.zeros(max(K, 1), np.uint8),
                 object_node=np.zeros(max(K, 1), np.int32), object_bbox=np.zeros((max(K, 1), 6), np.float64))
        self._check(self.L.mc_pp_get_results(self.h, _ptr(r["entry_object"]), _ptr(r["mask_object"]),
                                             _ptr(r["mask_coverage"]), _ptr(r["object_state"]), _ptr(r["object_node"]),
                                             _ptr(r["object_bbox"])))
        n = dict(entry_object=E, mask_object=Q, mask_coverage=Q, object_state=K, object_node=K, object_bbox=K)
        return {k: v[:n[k]] for k, v in r.items()}

    for f in (pp_run, pp_info, pp_results):
        setattr(Context, f.__name__, f)


_pp_methods()


def _eval_methods():
    def eval_match_counts(self, pred_masks, gt_instance, num_gt, void_flags):
        """evaluation/evaluate.py:289-308 on the device: (vert counts [K], void intersections [K],
        intersections [K, num_gt]) of the columns of pred_masks [P, K]."""
        pm = np.ascontiguousarray(np.asarray(pred_masks) != 0, np.uint8)
        P, K = pm.shape
        g = np.ascontiguousarray(gt_instance, np.int32)
        v = np.ascontiguousarray(void_flags, np.uint8)
        verts, vint = np.zeros(max(K, 1), np.int64), np.zeros(max(K, 1), np.int64)
        inter = np.zeros((max(K, 1), max(int(num_gt), 1)), np.int64)
        self._check(self.L.mc_eval_match_counts(self.h, P, K, _ptr(pm), _ptr(g), int(num_gt), _ptr(v), _ptr(verts),
                                                _ptr(vint), _ptr(inter)))
        return verts[:K], vint[:K], inter[:K, :int(num_gt)]

    Context.eval_match_counts = eval_match_counts


_eval_methods()


def _ov_methods():
    def openvoc_query(self, obj_off, obj_rows, features, label_features, temperature=100.0):
        """semantics/open-voc_query.py:32-50 on the device: label index of every object (-1: none)."""
        off = np.ascontiguousarray(obj_off, np.int64)
        rows = np.ascontiguousarray(obj_rows, np.int32)
        feats = np.ascontiguousarray(features, np.float32)
        labs = np.ascontiguousarray(label_features, np.float32)
        K = len(off) - 1
        out = np.zeros(max(K, 1), np.int32)
        self._check(self.L.mc_openvoc_query(self.h, K, _ptr(off), _ptr(rows), feats.shape[0], labs.shape[1],
                                            _ptr(feats), labs.shape[0], _ptr(labs), float(temperature), _ptr(out)))
        return out[:K]

    Context.openvoc_query = openvoc_query


_ov_methods()


def _io_methods():
    def frames_decode(self, num_frames, height, width, depth_ptr, depth_scale, seg_shape, seg_ptr, on_device,
                      depth_out_ptr, seg_out_ptr):
        """mc_frames_decode (dataset/scannet.py:49-54, :68-73); pointers as ints (None = skip)."""
        c = lambda x: None if x is None else ctypes.c_void_p(int(x))
        hs, ws = seg_shape
        self._check(self.L.mc_frames_decode(self.h, int(num_frames), int(height), int(width), c(depth_ptr),
                                            float(depth_scale), int(hs), int(ws), c(seg_ptr), 1 if on_device else 0,
                                            c(depth_out_ptr), c(seg_out_ptr)))

    Context.frames_decode = frames_decode


_io_methods()


def bits_unpack(words, ncols):
    """(R, W) little-endian uint64 bit rows -> (R, ncols) bool, unpacked by mc_bits_unpack's host
    threads (no GPU needed)."""
    words = np.ascontiguousarray(words, dtype="<u8")
    R = words.shape[0]
    out = np.empty((R, ncols), np.bool_)
    if R and ncols:
        rc = load().mc_bits_unpack(_ptr(words), R, words.shape[1], ncols, _ptr(out))
        if rc != 0:
            raise McError(rc, "mc_bits_unpack: bad sizes")
    return out
