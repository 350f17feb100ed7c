"""Python side of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Loads ``oracle/build/liboracle.so`` (built from ``mcgraph_oracle.c`` by
``oracle/Makefile``) and returns the outputs of the reference's graph stages
in the canonical form of the golden fixtures (``tests/golden/make_golden.py``):

* S2 ``build_point_in_mask_matrix`` — graph/construction.py:22-64
* S3 ``process_masks``              — graph/construction.py:137-170
* S4 ``get_observer_num_thresholds``— graph/construction.py:80-96
* S5 ``init_nodes``                 — graph/construction.py:66-78
* S6 ``iterative_clustering``       — graph/iterative_clustering.py:36-43

Only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may import this module.  The product library never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")
_lib = None

_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_i64p = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
_u16p = np.ctypeslib.ndpointer(np.uint16, flags="C_CONTIGUOUS")
_u64p = np.ctypeslib.ndpointer(np.uint64, flags="C_CONTIGUOUS")
_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


class BpParams(ctypes.Structure):
    """orc_bp_params (s1_oracle.c); defaults = the reference's constants
    (utils/mask_backprojection.py:8-14,38; utils/geometry.py:10,16,22)."""
    _fields_ = [("depth_trunc", ctypes.c_double), ("voxel_size", ctypes.c_double),
                ("dbscan_eps", ctypes.c_double), ("component_min_fraction", ctypes.c_double),
                ("sor_std_ratio", ctypes.c_double), ("ball_radius", ctypes.c_double),
                ("coverage_threshold", ctypes.c_double), ("dbscan_min_points", ctypes.c_int32),
                ("sor_neighbors", ctypes.c_int32), ("ball_k", ctypes.c_int32), ("few_points", ctypes.c_int32)]

    @classmethod
    def default(cls, **kw):
        p = cls(20.0, 0.01, 0.04, 0.2, 2.0, 0.01, 0.3, 4, 20, 20, 25)
        for k, v in kw.items():
            setattr(p, k, v)
        return p


S1_STATS = ["id", "npix", "nvox", "ndbscan", "nsor", "ncand", "ncovered", "nneighbors", "kept"]


def s1_frame(scene_f32, depth, seg, K, pose, params: BpParams | None = None):
    """turn_mask_to_point (utils/mask_backprojection.py:70-151) for one frame.
    Returns (labels int32 [n], off int64 [n+1], pts int32, stats int32 [n_cand, 9]).
    Raises IndexError where the reference does (a depth pixel == DEPTH_TRUNC)."""
    L = lib()
    prm = params or BpParams.default()
    scene = np.ascontiguousarray(scene_f32, np.float32).reshape(-1, 3)
    depth = np.ascontiguousarray(depth, np.float32)
    seg = np.ascontiguousarray(seg, np.uint8)
    H, W = depth.shape
    K = np.ascontiguousarray(K, np.float64).reshape(4)
    T = np.ascontiguousarray(pose, np.float64).reshape(16)
    labels = np.zeros(256, np.int32)
    off = np.zeros(257, np.int64)
    stats = np.zeros((256, len(S1_STATS)), np.int32)
    need = ctypes.c_int64()
    ncand = ctypes.c_int32()
    cap = 1 << 16
    while True:
        pts = np.zeros(cap, np.int32)
        n = L.orc_s1_frame(len(scene), scene.reshape(-1), H, W, depth.reshape(-1), seg.reshape(-1), K, T,
                           ctypes.byref(prm), labels, off, pts, cap, ctypes.byref(need), stats.reshape(-1),
                           ctypes.byref(ncand))
        if n == -2:
            cap = int(need.value)
            continue
        break
    if n == -1:
        raise IndexError("depth pixel equal to DEPTH_TRUNC (utils/mask_backprojection.py:100)")
    return labels[:n].copy(), off[:n + 1].copy(), pts[:off[n]].copy(), stats[:ncand.value].copy()


def s1_frames(scene_f32, depth, seg, K, poses, params: BpParams | None = None, threads: int | None = None):
    """s1_frame for many frames at once, OpenMP over frames (orc_s1_batch; frames are independent,
    utils/mask_backprojection.py:154-156).  depth / seg: sequences of [H,W] arrays (or [F,H,W]).
    Returns [(labels, off, pts, stats)] per frame, as s1_frame; IndexError for a DEPTH_TRUNC frame."""
    L = lib()
    prm = params or BpParams.default()
    scene = np.ascontiguousarray(scene_f32, np.float32).reshape(-1, 3)
    dl = [np.ascontiguousarray(d, np.float32) for d in depth]
    sl = [np.ascontiguousarray(x, np.uint8) for x in seg]
    F = len(dl)
    if F == 0:
        return []
    H, W = dl[0].shape
    assert all(d.shape == (H, W) and x.shape == (H, W) for d, x in zip(dl, sl))
    Kf = np.ascontiguousarray(K, np.float64).reshape(F, 4)
    Tf = np.ascontiguousarray(poses, np.float64).reshape(F, 16)
    dp = (ctypes.c_void_p * F)(*[d.ctypes.data for d in dl])
    sp = (ctypes.c_void_p * F)(*[x.ctypes.data for x in sl])
    n = np.zeros(F, np.int32)
    labels = np.zeros((F, 256), np.int32)
    off = np.zeros((F, 257), np.int64)
    stats = np.zeros((F, 256, len(S1_STATS)), np.int32)
    ncand = np.zeros(F, np.int32)
    total = ctypes.c_int64()
    h = L.orc_s1_batch(len(scene), scene.reshape(-1), F, H, W, dp, sp, Kf, Tf, ctypes.byref(prm),
                       int(threads or default_threads()), n, labels, off, stats, ncand, ctypes.byref(total))
    pts = np.zeros(max(int(total.value), 1), np.int32)
    L.orc_s1_batch_take(h, pts)
    out, o = [], 0
    for f in range(F):
        if n[f] == -1:
            raise IndexError(f"frame {f}: depth pixel equal to DEPTH_TRUNC (utils/mask_backprojection.py:100)")
        k = int(n[f])
        np_f = int(off[f, k])
        out.append((labels[f, :k].copy(), off[f, :k + 1].copy(), pts[o:o + np_f].copy(), stats[f, :ncand[f]].copy()))
        o += np_f
    return out


class threads:
    """``with oracle.threads(n):`` runs the OpenMP loops of the S2-S6 oracle on n threads"""

    def __init__(self, n: int):
        self.n = int(n)

    def __enter__(self):
        self.prev = lib().orc_num_threads()
        lib().orc_set_num_threads(self.n)
        return self

    def __exit__(self, *exc):
        lib().orc_set_num_threads(self.prev)


def default_threads() -> int:
    """host threads for the oracle: OMP_NUM_THREADS when set (16 per GPU on the box), else all cores"""
    return int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)


def s1_scene(frames, params: BpParams | None = None, timings: dict | None = None, threads: int | None = None):
    """All frames of a SceneFrames (maskclustering_amd.synthetic_frames) ->
    the flat mask CSR the graph stages consume (mask_col, mask_label, mask_off,
    mask_pts) plus the per-candidate stats with the frame column prepended."""
    scene = np.asarray(frames.scene_points, np.float64).astype(np.float32)  # construction.py:37
    cols, labs, offs, chunks, stats = [], [], [0], [], []
    t0 = time.perf_counter()
    res = s1_frames(scene, frames.depth, frames.seg, frames.intrinsics, frames.poses, params, threads)
    for f in range(frames.num_frames):
        lab, off, pts, st = res[f]
        for k in range(len(lab)):
            cols.append(f)
            labs.append(int(lab[k]))
            chunks.append(pts[off[k]:off[k + 1]])
            offs.append(offs[-1] + int(off[k + 1] - off[k]))
        stats.append(np.concatenate([np.full((len(st), 1), f, np.int32), st], axis=1))
    if timings is not None:
        timings["s1"] = time.perf_counter() - t0
    return dict(mask_col=np.asarray(cols, np.int32), mask_label=np.asarray(labs, np.int32),
                mask_off=np.asarray(offs, np.int64),
                mask_pts=np.concatenate(chunks).astype(np.int32) if chunks else np.zeros(0, np.int32),
                stats=np.concatenate(stats) if stats else np.zeros((0, len(S1_STATS) + 1), np.int32))


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.orc_s2.restype = ctypes.c_int
        L.orc_s2.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int, _i32p, _i32p, _i64p, _i32p,
                             _u8p, _u16p, _u8p, _u8p]
        L.orc_s3.restype = ctypes.c_int
        L.orc_s3.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int, _i32p, _i32p, _i64p, _i32p,
                             _u16p, _u8p, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                             _u8p, _i32p, _u8p]
        L.orc_observer_hist.restype = None
        L.orc_observer_hist.argtypes = [ctypes.c_int, ctypes.c_int, _u8p, _u64p]
        L.orc_thresholds.restype = ctypes.c_int
        L.orc_thresholds.argtypes = [_u64p, ctypes.c_int, _f32p, _i32p]
        L.orc_cluster.restype = ctypes.c_int
        L.orc_cluster.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _u8p, _u8p, ctypes.c_int, _f32p,
                                  ctypes.c_double, _i32p, _i32p, _i32p, _u8p, _u8p]
        L.orc_num_threads.restype = ctypes.c_int
        L.orc_set_num_threads.restype = None
        L.orc_set_num_threads.argtypes = [ctypes.c_int]
        L.orcs_s2.restype = ctypes.c_int
        L.orcs_s2.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int, _i32p, _i64p, _i32p, _u8p, _u8p, _i64p, _i32p]
        L.orcs_s3.restype = ctypes.c_int
        L.orcs_s3.argtypes = [ctypes.c_int, _i32p, _i32p, _i64p, _i32p, _u8p, _i32p, _u8p, _i64p, _i32p,
                              ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_int, _i32p, _i32p, _i32p,
                              _u8p, ctypes.c_void_p]
        L.orcs_undo.restype = None
        L.orcs_undo.argtypes = [ctypes.c_int, ctypes.c_int, _i32p, _i32p, _i32p, _u8p]
        L.orcs_observer_hist.restype = None
        L.orcs_observer_hist.argtypes = [ctypes.c_int, ctypes.c_int, _u64p, _u64p, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int]
        L.orcs_level_edges.restype = ctypes.c_int64
        L.orcs_level_edges.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _u64p, _i64p, _i32p, ctypes.c_float,
                                       ctypes.c_double, ctypes.c_int, ctypes.c_int, _i64p, ctypes.c_int64]
        L.orcs_cluster.restype = ctypes.c_int
        L.orcs_cluster.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _u64p, _i64p, _i32p, ctypes.c_int, _f32p,
                                   ctypes.c_double, _i32p, _i32p, _i32p, _i64p, _u64p, _i64p, _i32p]
        L.orcs_set_edge_sink.restype = None
        L.orcs_set_edge_sink.argtypes = [ctypes.c_void_p, ctypes.c_int64]
        L.orcs_edge_sink_count.restype = ctypes.c_int64
        L.orcs_edge_sink_count.argtypes = []
        _f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
        L.orc_s1_batch.restype = ctypes.c_void_p
        L.orc_s1_batch.argtypes = [ctypes.c_int64, _f32p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                   ctypes.c_void_p, _f64p, _f64p, ctypes.POINTER(BpParams), ctypes.c_int, _i32p, _i32p,
                                   _i64p, _i32p, _i32p, ctypes.POINTER(ctypes.c_int64)]
        L.orc_s1_batch_take.restype = None
        L.orc_s1_batch_take.argtypes = [ctypes.c_void_p, _i32p]
        L.orc_s1_frame.restype = ctypes.c_int
        L.orc_s1_frame.argtypes = [ctypes.c_int64, _f32p, ctypes.c_int, ctypes.c_int, _f32p, _u8p, _f64p, _f64p,
                                   ctypes.POINTER(BpParams), _i32p, _i64p, _i32p, ctypes.c_int64,
                                   ctypes.POINTER(ctypes.c_int64), _i32p, ctypes.POINTER(ctypes.c_int32)]
        _lib = L
    return _lib


def thresholds_from_hist(hist: np.ndarray):
    """numpy-2 float32 percentile ladder from an observer-count histogram."""
    hist = np.ascontiguousarray(hist, dtype=np.uint64)
    F = len(hist) - 1
    thr = np.zeros(20, np.float32)
    isint = np.zeros(20, np.int32)
    n = lib().orc_thresholds(hist, F, thr, isint)
    if n < 0:
        return None, None
    return thr[:n].copy(), isint[:n].astype(bool)


def observer_hist(vf: np.ndarray) -> np.ndarray:
    vf = np.ascontiguousarray(vf, dtype=np.uint8)
    M, F = vf.shape
    hist = np.zeros(F + 1, np.uint64)
    lib().orc_observer_hist(M, F, vf, hist)
    return hist


def cluster(vf0: np.ndarray, cm0: np.ndarray, thr: np.ndarray, ct: float):
    """S6 on explicit 0/1 node rows (bytes).  Returns (labels per iteration,
    level sizes, final label of each initial node, final vf, final cm)."""
    vf0 = np.ascontiguousarray(vf0, dtype=np.uint8)
    cm0 = np.ascontiguousarray(cm0, dtype=np.uint8)
    N0, F = vf0.shape
    M = cm0.shape[1]
    thr = np.ascontiguousarray(thr, dtype=np.float32)
    T = len(thr)
    labels = np.full((max(T, 1), max(N0, 1)), -1, np.int32)
    sizes = np.zeros(T + 1, np.int32)
    final = np.zeros(max(N0, 1), np.int32)
    vf_out = np.zeros((max(N0, 1), F), np.uint8)
    cm_out = np.zeros((max(N0, 1), M), np.uint8)
    K = lib().orc_cluster(N0, F, M, vf0, cm0, T, thr, float(ct), labels, sizes, final, vf_out, cm_out)
    parts = [labels[t, :sizes[t]].copy() for t in range(T)]
    return parts, sizes, final[:N0], vf_out[:K], cm_out[:K]


def run(num_points, num_frames, mask_col, mask_label, mask_off, mask_pts,
        mask_visible_threshold, undersegment_filter_threshold, view_consensus_threshold,
        contained_threshold, timings: dict | None = None):
    """Whole S2–S6 path on the CPU; returns the golden-fixture dictionary."""
    L = lib()
    P, F = int(num_points), int(num_frames)
    col = np.ascontiguousarray(mask_col, np.int32)
    label = np.ascontiguousarray(mask_label, np.int32)
    off = np.ascontiguousarray(mask_off, np.int64)
    pts = np.ascontiguousarray(mask_pts, np.int32)
    M_in = len(col)
    t0 = time.perf_counter()
    kept = np.zeros(max(M_in, 1), np.uint8)
    pim = np.zeros((P, F), np.uint16)
    pfm = np.zeros((P, F), np.uint8)
    bnd = np.zeros(P, np.uint8)
    M = L.orc_s2(P, F, M_in, col, label, off, pts, kept, pim, pfm, bnd)
    keep_idx = np.nonzero(kept[:M_in])[0]
    gcol, glabel = col[keep_idx], label[keep_idx]
    lens = (off[1:] - off[:-1])[keep_idx]
    goff = np.zeros(M + 1, np.int64)
    np.cumsum(lens, out=goff[1:])
    gpts = np.concatenate([pts[off[g]:off[g + 1]] for g in keep_idx]).astype(np.int32) if M else np.zeros(0, np.int32)
    t1 = time.perf_counter()
    vf = np.zeros((max(M, 1), F), np.uint8)
    ctgt = np.zeros((max(M, 1), F), np.int32)
    useg = np.zeros(max(M, 1), np.uint8)
    L.orc_s3(P, F, M, gcol, glabel, goff, gpts, pim, bnd, float(mask_visible_threshold),
             float(contained_threshold), float(undersegment_filter_threshold), vf, ctgt, useg)
    vf, ctgt, useg = vf[:M], ctgt[:M], useg[:M]
    t2 = time.perf_counter()
    hist = observer_hist(vf)
    thr, thr_isint = thresholds_from_hist(hist)
    t3 = time.perf_counter()
    if thr is None:
        raise IndexError("no positive observer count (np.percentile of an empty array)")
    node0 = np.nonzero(useg == 0)[0].astype(np.int32)
    cm = np.zeros((len(node0), M), np.uint8)
    r, c = np.nonzero(ctgt[node0] >= 0)
    cm[r, ctgt[node0][r, c]] = 1
    t4 = time.perf_counter()
    parts, sizes, final, fvf, fcm = cluster(vf[node0], cm, thr, float(view_consensus_threshold))
    t5 = time.perf_counter()
    if timings is not None:
        timings.update(s2=t1 - t0, s3=t2 - t1, s4=t3 - t2, s6=t5 - t4,
                       pairs=int(sum(int(s) ** 2 for s in sizes[:-1])) if len(thr) else 0,
                       threads=L.orc_num_threads())

    out = {}
    out["gl_col"], out["gl_label"] = gcol.copy(), glabel.copy()
    out["boundary"] = np.nonzero(bnd)[0].astype(np.int32)
    nzp, nzc = np.nonzero(pim)
    out["pim_p"], out["pim_c"], out["pim_v"] = nzp.astype(np.int32), nzc.astype(np.int32), pim[nzp, nzc].astype(np.int32)
    out["pfm_bits"] = np.packbits(pfm.astype(bool), axis=1)
    out["vf_bits"] = np.packbits(vf.astype(bool), axis=1)
    rr, cc = np.nonzero(ctgt >= 0)
    crow, ccol = rr.astype(np.int32), ctgt[rr, cc].astype(np.int32)
    order = np.lexsort((ccol, crow))
    out["c_row"], out["c_col"] = crow[order], ccol[order]
    out["undersegment"] = np.nonzero(useg)[0].astype(np.int32)
    out["thr_value"], out["thr_is_int"] = thr, thr_isint
    out["node0_g"] = node0
    T = len(thr)
    out["num_iters"] = np.array(T, np.int32)
    for t in range(T):
        out[f"part_{t}"] = parts[t]
    K = len(fvf)
    members = [[] for _ in range(K)]
    for i, k in enumerate(final):
        members[k].append(int(node0[i]))
    mo, mi, po, pi_, co, ci = [0], [], [0], [], [0], []
    for k in range(K):
        gs = sorted(members[k])
        mi.extend(gs); mo.append(len(mi))
        u = np.unique(np.concatenate([gpts[goff[g]:goff[g + 1]] for g in gs])) if gs else np.zeros(0, np.int32)
        pi_.extend(u.tolist()); po.append(len(pi_))
        cidx = np.nonzero(fcm[k])[0]
        ci.extend(cidx.tolist()); co.append(len(ci))
    out["obj_mask_off"], out["obj_mask_idx"] = np.array(mo, np.int64), np.array(mi, np.int32)
    out["obj_pt_off"], out["obj_pt_idx"] = np.array(po, np.int64), np.array(pi_, np.int32)
    out["obj_vf_bits"] = np.packbits(fvf.astype(bool), axis=1)
    out["obj_c_off"], out["obj_c_idx"] = np.array(co, np.int64), np.array(ci, np.int32)
    out["obj_node_info"] = np.array([(T, k) if T else (0, k) for k in range(K)], np.int32).reshape(-1, 2)
    if T:
        last = parts[T - 1]
        sons = [np.nonzero(last == k)[0].astype(np.int32) for k in range(K)]
    else:
        sons = [np.zeros(0, np.int32) for _ in range(K)]
    so = np.zeros(K + 1, np.int64)
    so[1:] = np.cumsum([len(s) for s in sons])
    out["obj_son_off"] = so
    out["obj_son_idx"] = np.concatenate(sons).astype(np.int32) if K else np.zeros(0, np.int32)
    return out


def _bits_rows(cols_per_row, n_rows, F):
    """rows of frame indices -> (n_rows, ceil(F/64)) uint64 little-endian bits"""
    FW = max((F + 63) // 64, 1)
    out = np.zeros((max(n_rows, 1), FW), np.uint64)
    for r, cs in enumerate(cols_per_row):
        if len(cs):
            np.bitwise_or.at(out[r], np.asarray(cs) // 64, np.left_shift(np.uint64(1), (np.asarray(cs) % 64).astype(np.uint64)))
    return out[:n_rows]


def run_sparse(num_points, num_frames, mask_col, mask_label, mask_off, mask_pts,
               mask_visible_threshold, undersegment_filter_threshold, view_consensus_threshold,
               contained_threshold, timings: dict | None = None, edge_cap: int = 0):
    """Whole S2-S6 path on the CPU with sparse rows (oracle/graph_sparse.c): the golden-fixture
    dictionary of run() without the dense point-in-mask entries (pim_*), for C3/C4-sized scenes.
    edge_cap > 0 also returns every S6 iteration's edges as out["edges"] = (t, a, b) sorted."""
    L = lib()
    if edge_cap > 0:
        sink = np.zeros(int(edge_cap), np.uint64)
        L.orcs_set_edge_sink(sink.ctypes.data, int(edge_cap))
        try:
            out = run_sparse(num_points, num_frames, mask_col, mask_label, mask_off, mask_pts,
                             mask_visible_threshold, undersegment_filter_threshold, view_consensus_threshold,
                             contained_threshold, timings)
            n = L.orcs_edge_sink_count()
        finally:
            L.orcs_set_edge_sink(None, 0)
        if n > edge_cap:
            raise ValueError(f"{n} edges exceed edge_cap {edge_cap}")
        k = np.sort(sink[:n])
        out["edges"] = ((k >> np.uint64(48)).astype(np.int64), ((k >> np.uint64(24)) & np.uint64(0xFFFFFF)).astype(np.int64),
                        (k & np.uint64(0xFFFFFF)).astype(np.int64))
        return out
    P, F = int(num_points), int(num_frames)
    col = np.ascontiguousarray(mask_col, np.int32)
    label = np.ascontiguousarray(mask_label, np.int32)
    off = np.ascontiguousarray(mask_off, np.int64)
    pts = np.ascontiguousarray(mask_pts, np.int32)
    M_in = len(col)
    t0 = time.perf_counter()
    kept = np.zeros(max(M_in, 1), np.uint8)
    bnd = np.zeros(max(P, 1), np.uint8)
    pt_off = np.zeros(P + 1, np.int64)
    pt_ent = np.zeros(max(int(off[-1]) if M_in else 0, 1), np.int32)
    M = L.orcs_s2(P, F, M_in, col, off, pts, kept, bnd, pt_off, pt_ent)
    kept = kept[:M_in]
    gidx = np.where(kept > 0, np.cumsum(kept) - 1, -1).astype(np.int32)
    t1 = time.perf_counter()
    Fc = max(F, 1)
    ct_frame = np.zeros(max(M, 1) * Fc, np.int32)
    ct_tgt = np.zeros(max(M, 1) * Fc, np.int32)
    ct_len = np.zeros(max(M, 1), np.int32)
    useg = np.zeros(max(M, 1), np.uint8)
    L.orcs_s3(M_in, col, label, off, pts, np.ascontiguousarray(kept), gidx, bnd, pt_off, pt_ent,
              float(mask_visible_threshold), float(contained_threshold), float(undersegment_filter_threshold), Fc,
              ct_frame, ct_tgt, ct_len, useg, None)
    L.orcs_undo(M, Fc, ct_frame, ct_tgt, ct_len, useg)
    ct_frame, ct_tgt = ct_frame.reshape(-1, Fc), ct_tgt.reshape(-1, Fc)
    ct_len, useg = ct_len[:M], useg[:M]
    FW = max((F + 63) // 64, 1)
    rr = np.repeat(np.arange(M), ct_len)
    cc = np.concatenate([ct_frame[r, :ct_len[r]] for r in range(M)]) if M else np.zeros(0, np.int32)
    tt = np.concatenate([ct_tgt[r, :ct_len[r]] for r in range(M)]) if M else np.zeros(0, np.int32)
    vfw = np.zeros((max(M, 1), FW), np.uint64)
    if len(rr):
        np.bitwise_or.at(vfw, (rr, cc // 64), np.left_shift(np.uint64(1), (cc % 64).astype(np.uint64)))
    vfw = np.ascontiguousarray(vfw[:M] if M else vfw)
    t2 = time.perf_counter()
    hist = np.zeros(F + 1, np.uint64)
    L.orcs_observer_hist(M, FW, vfw, hist, F, 0, 1)
    thr, thr_isint = thresholds_from_hist(hist)
    t3 = time.perf_counter()
    if thr is None:
        raise IndexError("no positive observer count (np.percentile of an empty array)")
    node0 = np.nonzero(useg == 0)[0].astype(np.int32)
    order = np.lexsort((tt, rr))
    rr_s, tt_s = rr[order], tt[order]
    c_off_all = np.zeros(M + 1, np.int64)
    np.cumsum(ct_len, out=c_off_all[1:])
    lens0 = ct_len[node0].astype(np.int64)
    c_off0 = np.zeros(len(node0) + 1, np.int64)
    np.cumsum(lens0, out=c_off0[1:])
    c_idx0 = np.concatenate([tt_s[c_off_all[g]:c_off_all[g + 1]] for g in node0]).astype(np.int32) \
        if len(node0) and c_off0[-1] else np.zeros(1, np.int32)
    N0 = len(node0)
    T = len(thr)
    labels = np.full((max(T, 1), max(N0, 1)), -1, np.int32)
    sizes = np.zeros(T + 1, np.int32)
    final = np.zeros(max(N0, 1), np.int32)
    edges = np.zeros(max(T, 1), np.int64)
    vf_out = np.zeros((max(N0, 1), FW), np.uint64)
    co_out = np.zeros(max(N0, 1) + 1, np.int64)
    ci_out = np.zeros(max(int(c_off0[-1]), 1), np.int32)
    t4 = time.perf_counter()
    K = L.orcs_cluster(N0, FW, M, np.ascontiguousarray(vfw[node0]) if N0 else np.zeros((1, FW), np.uint64), c_off0,
                       np.ascontiguousarray(c_idx0), T, np.ascontiguousarray(thr, np.float32),
                       float(view_consensus_threshold), labels, sizes, final, edges, vf_out, co_out, ci_out)
    t5 = time.perf_counter()
    if timings is not None:
        timings.update(s2=t1 - t0, s3=t2 - t1, s4=t3 - t2, s6=t5 - t4,
                       pairs=int(sum(int(s) ** 2 for s in sizes[:-1])) if T else 0, threads=L.orc_num_threads())
    return assemble_sparse(P, F, col, label, off, pts, kept, bnd, rr, tt, useg, vfw, hist, thr, thr_isint, node0,
                           [labels[t, :sizes[t]].copy() for t in range(T)], sizes, final[:N0], edges[:T],
                           vf_out[:K], co_out[:K + 1], ci_out[:co_out[K]])


def assemble_sparse(P, F, col, label, off, pts, kept, bnd, c_rows, c_tgts, useg, vfw, hist, thr, thr_isint, node0,
                    parts, sizes, final, edges, vf_fin, c_off_fin, c_idx_fin):
    """The golden-fixture dictionary (without pim_*) from the sparse stages' pieces: c_rows / c_tgts
    = the contained entries (row, target global mask) after the undo, any order."""
    M = int(np.count_nonzero(kept))
    T = len(parts)
    K = len(c_off_fin) - 1
    order = np.lexsort((c_tgts, c_rows))
    rr_s, tt_s = np.asarray(c_rows)[order], np.asarray(c_tgts)[order]
    N0 = len(node0)
    out = {}
    keep_idx = np.nonzero(kept)[0]
    out["gl_col"], out["gl_label"] = col[keep_idx].copy(), label[keep_idx].copy()
    out["boundary"] = np.nonzero(bnd[:P])[0].astype(np.int32)
    out["vf_bits"] = np.packbits(_bits_to_bool(vfw, F), axis=1) if M else np.zeros((0, (F + 7) // 8), np.uint8)
    out["c_row"], out["c_col"] = rr_s.astype(np.int32), tt_s.astype(np.int32)
    out["undersegment"] = np.nonzero(useg)[0].astype(np.int32)
    out["thr_value"], out["thr_is_int"] = thr, thr_isint
    out["node0_g"] = node0
    out["observer_hist"] = hist
    out["num_iters"] = np.array(T, np.int32)
    out["level_sizes"] = sizes
    out["edge_counts"] = np.asarray(edges, np.int64)[:T].copy()
    for t in range(T):
        out[f"part_{t}"] = np.asarray(parts[t], np.int32)
    fin = np.asarray(final)[:N0]
    order = np.argsort(fin, kind="stable")
    mo = np.zeros(K + 1, np.int64)
    np.cumsum(np.bincount(fin, minlength=K), out=mo[1:])
    out["obj_mask_off"], out["obj_mask_idx"] = mo, node0[order].astype(np.int32)
    # object points: union of the member masks' point sets (node.py:35), ascending
    goff = np.zeros(M + 1, np.int64)
    np.cumsum((off[1:] - off[:-1])[keep_idx], out=goff[1:])
    obj_of_g = np.full(M, -1, np.int64)
    obj_of_g[node0] = fin
    gl_pts = np.concatenate([pts[off[g]:off[g + 1]] for g in keep_idx]).astype(np.int64) if M else np.zeros(0, np.int64)
    og = np.repeat(obj_of_g, np.diff(goff))
    sel = og >= 0
    key = np.unique(og[sel] * max(P, 1) + gl_pts[sel])
    ko = key // max(P, 1)
    po = np.zeros(K + 1, np.int64)
    np.cumsum(np.bincount(ko, minlength=K), out=po[1:])
    out["obj_pt_off"], out["obj_pt_idx"] = po, (key % max(P, 1)).astype(np.int32)
    out["obj_vf_bits"] = np.packbits(_bits_to_bool(vf_fin, F), axis=1) if K else np.zeros((0, (F + 7) // 8), np.uint8)
    out["obj_c_off"], out["obj_c_idx"] = np.asarray(c_off_fin, np.int64).copy(), np.asarray(c_idx_fin, np.int32).copy()
    out["obj_node_info"] = np.array([(T, k) if T else (0, k) for k in range(K)], np.int32).reshape(-1, 2)
    if T:
        last = np.asarray(parts[T - 1])
        so = np.zeros(K + 1, np.int64)
        np.cumsum(np.bincount(last, minlength=K), out=so[1:])
        out["obj_son_off"], out["obj_son_idx"] = so, np.argsort(last, kind="stable").astype(np.int32)
    else:
        out["obj_son_off"], out["obj_son_idx"] = np.zeros(K + 1, np.int64), np.zeros(0, np.int32)
    return out


def _bits_to_bool(words, n):
    words = np.ascontiguousarray(words, dtype="<u8")
    if words.size == 0:
        return np.zeros((words.shape[0], n), bool)
    b = np.unpackbits(words.view(np.uint8).reshape(words.shape[0], -1), axis=1, bitorder="little")
    return b[:, :n].astype(bool)
