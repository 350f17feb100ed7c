"""Benchmark of the view-consensus graph path on MI355X.

A step = one pass of the hot path over one synthetic scene.  Default: the ScanNet++-shaped C3 scene
(BASELINE.json configs[2]: 1500 frames 1920x1440, ~1M points, ~80k masks), end to end:

  --variant e2e (default) S1 back-projection of every frame from depth / segmentation / poses
                resident in HBM, then graph construction S2-S5 and iterative clustering S6 to the
                final per-object point sets;
  --variant g   S2-S6 only, from per-frame mask sets resident in HBM;
  --variant pp / api / sweep: the post-processing row, the reference-API call sequence of
                main.py:17-21, and the 312-scene sweep (BASELINE configs[4]), each its own line.

metric: mask-pair consensus counts/sec = Σ_t N_t² (the ordered node pairs whose view consensus
the reference evaluates, graph/iterative_clustering.py:20-29) per scene × scenes ÷ max-over-ranks
wall time; ms_per_step is the per-scene graph build + cluster time (BASELINE.json's first metric).
Multi-GPU (--shard frames, default): one scene per step, its frames split over the ranks (strong
scaling); --shard scene: every rank its own scene (weak scaling, run.py:33-50).
At N=1 the line also carries `secondary`: the ScanNet-sized C2 scene (configs[1]) timed E2E and G
in the same process, with the host ports beside it (c2_record).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--variant e2e|g|pp|api|sweep] [--shape S]
                    [--no-cpu-baseline] [--no-secondary]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from types import SimpleNamespace

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
import maskclustering_amd  # noqa: E402,F401  (HIP queue setting before the first HIP call)

HBM_PEAK_GBS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md)
INT8_MFMA_PEAK_TOPS = 5000.0  # dense int8 MFMA (2x the 2.5 PF bf16 dense)
from maskclustering_amd.dataset_configs import DATASET_THRESHOLDS, shape_thresholds  # noqa: E402

# the graph thresholds of the reference's configs/scannet.json (C2, the ScanNet-shaped scene); every
# step runs under its shape's own dataset config (shape_thresholds: C3 = configs/scannetpp.json)
CFG = shape_thresholds("c2")[1]
G_GROUPS = ["s2_point_lists", "s3_masks", "s3_undo_s5", "s4_observer_hist", "s6_columns", "s6_pairs",
            "s6_components", "s6_merge", "s7_points"]
BP_GROUPS = ["bp_grid", "bp_pixels", "bp_voxel", "bp_denoise", "bp_query"]


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def own_device_budget(ctx, share=0.65):
    """The bench owns its device: S1's batches may take `share` of the free HBM (the library's
    default for callers that share the device is 40 % of it at most, mc_ctx_set_memory_budget)."""
    import torch
    free, _ = torch.cuda.mem_get_info()
    ctx.set_memory_budget(int(free * share))


def graph_work(ctx, mask_pts, P, F):
    """Per-launch algorithmic work of every graph kernel group.

    Returns {group: (bound, per_launch, model, alt)}: the primary model is SURVEY.md §8(d)'s
    where it defines one (S2, S3: dense-equivalent bytes of the reference's point-in-mask
    matrix; S4, S6: dense-equivalent int8 MFMA ops 2·N²·K), so a sparse kernel can exceed 1;
    ``alt`` is the builder's minimal-bytes model of what the sparse kernel must touch."""
    gi = ctx.graph_info()
    ci = ctx.cluster_info()
    M, nnz = gi.num_masks, len(mask_pts)
    FW = (F + 63) // 64
    deg = np.bincount(mask_pts, minlength=P).astype(np.int64)
    bnd = ctx.boundary(P).astype(bool)
    nb = ~bnd[mask_pts]
    nvalid = int(nb.sum())
    nnzC = int(gi.num_contained)
    T = int(ci.num_iterations)
    N = ctx.level_sizes(T).astype(np.float64)
    cap = ctx.level_caps(T).astype(np.float64)
    w = {}
    # S2 (§8(d)): 2·P·F + P·F/8 + 4·Σ|m|  |  alt: read ids, write + sort point lists, offsets,
    # boundary, point-frame bits
    w["s2_point_lists"] = ("hbm", float(2 * P * F + P * F / 8 + 4 * nnz), "SURVEY §8(d) S2 dense-equivalent bytes",
                           float(4 * nnz + 16 * nnz + 9 * P + 8 * P * FW))
    # S3 (§8(d)): 2·F·Σ|valid_m| + 4·Σ|m| + M·F/8  |  alt: ids + boundary flags of every mask point,
    # offsets + list entries of every non-boundary point, contained rows + flags
    w["s3_masks"] = ("hbm", float(2 * F * nvalid + 4 * nnz + M * F / 8), "SURVEY §8(d) S3 dense-equivalent bytes",
                     float(8 * M + 5 * nnz + int(np.sum(8 + 4 * deg[mask_pts[nb]])) + 4 * nnzC + 5 * M))
    # undo + S5: contained rows read twice and written once, VF rows, node arrays
    w["s3_undo_s5"] = ("hbm", float(12 * nnzC + 16 * FW * M + 40 * M), "contained rows r/w, VF, node arrays", None)
    # S4: observer GEMM VF·VFᵀ over all M masks (construction.py:84) as int8 MFMA ops
    w["s4_observer_hist"] = ("mfma", 2.0 * M * M * F, "SURVEY §8(d) 2·M²·F dense-equivalent int8 ops", None)
    if T:
        # S6 per iteration t (§8(d)): 2·N_t²·(F+M) dense-equivalent int8 ops, averaged over the T launches
        w["s6_pairs"] = ("mfma", float(np.sum(2.0 * N[:T] ** 2 * (F + M)) / T),
                         "SURVEY §8(d) Σ_t 2·N_t²·(F+M) / T dense-equivalent int8 ops", None)
        # components: parents read, roots / labels / level labels / member lists written, member
        # counts; offsets of the next level
        w["s6_components"] = ("hbm", float(np.sum(24 * N[:T] + 8 * N[1:T + 1]) / T),
                              "24·N_t + 8·N_(t+1) bytes per iteration", None)
        # merge: members' contained rows (<= cap_t slots) + VF rows read, new rows + owners + VF
        # written, plus the next level's column lists (read, relabel, write) on all but the last
        col = np.array([12.0 * nnzC if t + 1 < T else 0.0 for t in range(T)])
        w["s6_merge"] = ("hbm", float(np.sum(4 * cap[:T] + (8 * FW + 4) * N[:T] + 8 * cap[1:T + 1]
                                             + (8 * FW + 8) * N[1:T + 1] + col) / T),
                         "4·cap_t + (8·FW+4)·N_t + 8·cap_(t+1) + (8·FW+8)·N_(t+1) + 12·nnzC bytes per iteration",
                         None)
        w["s6_columns"] = ("hbm", float(20 * cap[0]), "level-0 transpose: 20·nnzC0 bytes", None)
    w["s7_points"] = ("hbm", float(2 * 4 * nnz + 4 * int(ci.num_object_points)), "8·nnz + 4·Σ|object points|", None)
    return w


def roofline_entry(w, avg_s, pmc_group=None):
    """Roofline of one kernel group: algorithmic work per launch (w = graph_work / bp_work
    entry) over its average launch duration avg_s; traffic = PMC HBM bytes per launch."""
    bound, per_launch, model, alt = w
    if bound == "hbm":
        achieved, peak, unit = per_launch / avg_s / 1e9, HBM_PEAK_GBS, "GB/s"
    else:
        achieved, peak, unit = per_launch / avg_s / 1e12, INT8_MFMA_PEAK_TOPS, "TFLOP/s"
    e = {"bound": bound, "achieved": round(achieved, 2), "peak": peak, "unit": unit, "frac": round(achieved / peak, 4),
         "traffic": None, "avg_launch_ms": round(avg_s * 1e3, 5), "algorithmic_per_launch": per_launch, "model": model}
    if bound == "mfma":
        e["note"] = ("dense-equivalent int8 ops of the reference's fp32 GEMMs; the kernel is sparse (it never "
                     "evaluates pairs with no shared contained mask), so frac can exceed 1 and says nothing "
                     "about efficiency: see traffic_frac_hbm")
    if alt is not None:
        e["alt_model_bytes"] = alt
        e["alt_frac"] = round(alt / avg_s / 1e9 / HBM_PEAK_GBS, 4)
    if pmc_group:
        t = float(pmc_group["bytes_per_launch"])
        e["traffic"] = round(t, 0)
        e["traffic_gbs"] = round(t / avg_s / 1e9, 2)
        e["traffic_frac_hbm"] = round(t / avg_s / 1e9 / HBM_PEAK_GBS, 4)
    return e


# the SQ counter passes of the benched build (scripts/gpu_final.sh PART=profiles); round 5's as a fallback
SQ_DENOISE = next((p for p in (os.path.join(REPO, "profiles", "r06", "final", "denoise_sq_counters_c3.json"),
                               os.path.join(REPO, "profiles", "r05", "denoise_sq_counters_c3.json"))
                   if os.path.exists(p)), os.path.join(REPO, "profiles", "r06", "final", "denoise_sq_counters_c3.json"))
SQ_DENOISE_FRAMES = 100     # the counter pass: C3 frames 600-699 (scripts/pmc_kernel.py over scripts/bp_profile.py)
CLOCK_GHZ = 2.4             # MI355X engine clock (MI355X_MICROARCH.md)


def denoise_valu(frames, launches, avg_s, voxels=None):
    """The denoise's second bound: VALU issue.  The committed SQ pass gives the size classes' VALU
    instructions per frame; times the frames of one launch (a batch), x 4 cycles per wave64
    instruction (a SIMD is 16 lanes wide), over the SIMDs' cycles in the live launch time."""
    if not os.path.exists(SQ_DENOISE):
        return None
    sq = json.load(open(SQ_DENOISE))
    ks = {k: v for k, v in sq.items() if "k_bp_denoise" in k or "k_bp_knn_ring" in k}
    insts = sum(v.get("SQ_INSTS_VALU", 0.0) for v in ks.values())
    simds = 4 * _torch_cu_count()
    per_launch = insts / SQ_DENOISE_FRAMES * frames / max(launches, 1)
    frac = per_launch * 4 / (simds * CLOCK_GHZ * 1e9 * avg_s)
    out = {"bound": "valu-issue", "insts_per_launch": round(per_launch, 0), "frac": round(frac, 4),
           "simds": simds, "clock_ghz": CLOCK_GHZ, "source": os.path.relpath(SQ_DENOISE, REPO),
           "note": "VALU instructions of the group's kernels per frame from the committed SQ counter pass of the "
                   "benched build, x the launch's frames, 4 cycles per wave64 instruction; the rest of the cycles "
                   "the waves wait on memory or barriers (SQ_WAIT_ANY / SQ_WAVE_CYCLES per kernel below)"}
    per = {}
    for k, v in ks.items():
        e = {}
        if v.get("SQ_WAVE_CYCLES"):
            e["wait_frac"] = round(v.get("SQ_WAIT_ANY", 0.0) / v["SQ_WAVE_CYCLES"], 3)
        if v.get("SQ_LDS_IDX_ACTIVE"):
            e["lds_bank_conflict_frac"] = round(v.get("SQ_LDS_BANK_CONFLICT", 0.0) / v["SQ_LDS_IDX_ACTIVE"], 3)
        if e:
            per[k.replace("mc::", "")] = e
    if per:
        out["per_kernel"] = per
    if voxels:  # the scene's voxels (denoise inputs) per launch
        out["insts_per_voxel"] = round(per_launch / (voxels / max(launches, 1)), 1)
        out["insts_per_voxel_note"] = "wave64 VALU instructions per input voxel (the SQ pass's frames scaled to the launch)"
    return out


def _torch_cu_count():
    import torch
    return int(torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count)


def bp_work(ctx, F, H, W):
    """Per-launch algorithmic bytes of the S1 groups: each frame's depth + seg
    read once and every mask pixel listed once (pixels); every mask pixel's list entry and
    depth read, every voxel written (voxel); voxels read, float32 mask points written
    (denoise); mask points read, neighbour ids written (query)."""
    st = ctx.bp_candidates()
    npx, nvox, nsor = int(st[:, 2].sum()), int(st[:, 3].sum()), int(st[:, 5].sum())
    nnbr = int(ctx.bp_info().num_mask_points)
    return {
        "bp_pixels": ("hbm", float(5 * F * H * W + 4 * npx), "5·F·H·W + 4·Σ mask pixels", None),
        "bp_voxel": ("hbm", float(8 * npx + 24 * nvox), "8·Σ mask pixels + 24·Σ voxels", None),
        "bp_denoise": ("hbm", float(24 * nvox + 12 * nsor), "24·Σ voxels + 12·Σ surviving points", None),
        "bp_query": ("hbm", float(12 * nsor + 4 * nnbr), "12·Σ mask points + 4·Σ neighbour ids", None),
    }


def s1_cpu_rate(scene_f32, frame_at, F, n_all=64, n_one=8):
    """Seconds per frame of the S1 port (oracle/s1_oracle.c) on the host: all threads (OpenMP over
    frames) on n_all frames spread evenly over the scene, and one thread on n_one of those frames.
    frame_at(i) -> (depth [H,W] f32, seg [H,W] u8, K [4], pose [4,4]) host arrays."""
    from oracle import oracle
    idx = np.unique(np.linspace(0, F - 1, min(n_all, F)).round().astype(np.int64))
    fr = [frame_at(int(i)) for i in idx]
    thr = oracle.default_threads()

    crop = []

    def timed(sel, threads):
        t0 = time.perf_counter()
        out = oracle.s1_frames(scene_f32, [fr[k][0] for k in sel], [fr[k][1] for k in sel],
                               np.stack([fr[k][2] for k in sel]), np.stack([fr[k][3] for k in sel]), threads=threads)
        dt = (time.perf_counter() - t0) / len(sel)
        if not crop:  # the reference's crop (crop_scene_points, :59-66) per mask that reaches it: stats "ncand"
            c = oracle.S1_STATS.index("ncand")
            crop.append(sum(int(st[:, c].sum()) for _, _, _, st in out) / len(sel))
        return dt

    one = list(range(0, len(idx), max(1, len(idx) // n_one)))[:n_one]
    return dict(all=timed(range(len(idx)), thr), one=timed(one, 1), threads=thr, n_all=len(idx), n_one=len(one),
                frames=F, crop_candidates_per_frame=crop[0])


def graph_cpu(P, F, col, lab, off, pts, threads, dense=False, cfg=None):
    """the S2-S6 port on `threads` host threads under thresholds `cfg` (default C2's): (seconds, timings)"""
    from oracle import oracle
    tm = {}
    with oracle.threads(threads):
        (oracle.run if dense else oracle.run_sparse)(P, F, col, lab, off, pts, timings=tm, **(cfg or CFG))
    return tm["s2"] + tm["s3"] + tm["s4"] + tm["s6"], tm


def e2e_cpu_baseline(s1, P, F, col, lab, off, pts, cfg):
    """cpu_baseline of the E2E variants: S1 port (per-frame rates of s1_cpu_rate x F frames) + the
    S2-S6 port on the full mask set, on all host threads (value) and on one (single_thread)."""
    g_all, tm = graph_cpu(P, F, col, lab, off, pts, s1["threads"], cfg=cfg)
    g_one, _ = graph_cpu(P, F, col, lab, off, pts, 1, cfg=cfg)
    all_s, one_s = s1["all"] * F + g_all, s1["one"] * F + g_one
    pairs = tm["pairs"]
    return {"value": round(pairs / all_s, 1), "unit": "mask-pairs/s", "cores": s1["threads"], "kind": "port",
            "s1_crop_candidates_per_frame": round(s1["crop_candidates_per_frame"], 1),
            "sample": f"S1 port (oracle/s1_oracle.c, OpenMP over frames, {s1['threads']} threads) timed on "
                      f"{s1['n_all']} frames spread over the {F} and scaled to {F} ({s1['all'] * F:.1f} s) + the "
                      f"S2-S6 port (oracle/graph_sparse.c, {s1['threads']} threads) on the full scene ({g_all:.2f} s)",
            "scene_ms": round(all_s * 1e3, 1),
            "single_thread": {"value": round(pairs / one_s, 1), "cores": 1, "scene_ms": round(one_s * 1e3, 1),
                              "sample": f"S1 port on 1 thread, {s1['n_one']} of those frames ({s1['one'] * F:.1f} s "
                                        f"scaled) + the S2-S6 port on 1 thread ({g_one:.2f} s)"}}


class GraphStep:
    """--variant g: per-frame mask sets resident in HBM -> final objects."""

    def __init__(self, shape, seed, local):
        import torch
        from maskclustering_amd.pipeline import GraphRun
        from maskclustering_amd.synthetic import SHAPES, make_shape
        self.scene = make_shape(shape, seed=seed)
        self.dataset, self.cfg = shape_thresholds(shape)
        self.run = GraphRun(local)
        self.run.ctx.set_stream(torch.cuda.current_stream().cuda_stream)
        self.run.set_scene(self.scene)
        self.groups = G_GROUPS
        sh = SHAPES[shape]
        self.workload = (f"{shape}: ScanNet-shaped synthetic scene (SURVEY App. C), P={sh['num_points']} "
                         f"F={sh['num_frames']}")

    def step(self):
        self.run.step(**self.cfg)

    def work(self):
        s = self.scene
        return graph_work(self.run.ctx, s.mask_pts, s.num_points, s.num_frames)

    def cpu_baseline(self):
        from oracle import oracle
        s = self.scene
        dense = s.num_masks <= 30000  # dense matrices beyond C2 do not fit
        thr = oracle.default_threads()
        masks = (s.mask_col, s.mask_label, s.mask_off, s.mask_pts)
        cpu_s, tm = graph_cpu(s.num_points, s.num_frames, *masks, thr, dense, cfg=self.cfg)
        one_s, _ = graph_cpu(s.num_points, s.num_frames, *masks, 1, dense, cfg=self.cfg)
        return {"value": round(tm["pairs"] / cpu_s, 1), "unit": "mask-pairs/s", "cores": thr, "kind": "port",
                "sample": f"{'oracle/mcgraph_oracle.c' if dense else 'oracle/graph_sparse.c'} S2-S6 on "
                          f"the same scene (1 full scene, {thr} threads, {cpu_s:.2f} s: "
                          f"S2 {tm['s2']:.2f} S3 {tm['s3']:.2f} S4 {tm['s4']:.2f} S6 {tm['s6']:.2f})",
                "scene_ms": round(cpu_s * 1e3, 1),
                "single_thread": {"value": round(tm["pairs"] / one_s, 1), "cores": 1, "scene_ms": round(one_s * 1e3, 1),
                                  "sample": "the same port and scene on 1 thread"}}


class EndToEndStep:
    """--variant e2e: depth / seg / poses resident in HBM -> back-projected masks -> final objects."""

    def __init__(self, shape, seed, local):
        import torch
        from maskclustering_amd import _native
        from maskclustering_amd.pipeline import GraphRun
        from maskclustering_amd.synthetic_frames import make_frames_shape
        t0 = time.perf_counter()
        fr = make_frames_shape(shape, seed=seed, device=f"cuda:{local}", out="torch")
        log(f"rendered {fr.num_frames} frames {fr.depth.shape[1]}x{fr.depth.shape[2]} P={fr.num_points} "
            f"in {time.perf_counter() - t0:.1f} s")
        self.fr = fr
        self.dataset, self.cfg = shape_thresholds(shape)
        dev = torch.device("cuda", local)
        self.t_scene = torch.tensor(fr.scene_points, dtype=torch.float32, device=dev)  # construction.py:37
        self.t_depth = fr.depth
        self.t_seg = fr.seg
        self.t_K = torch.from_numpy(np.ascontiguousarray(fr.intrinsics)).to(dev)
        self.t_T = torch.from_numpy(np.ascontiguousarray(fr.poses.reshape(-1, 16))).to(dev)
        self.run = GraphRun(local)
        self.ctx = self.run.ctx
        self.ctx.set_stream(torch.cuda.current_stream().cuda_stream)
        self.ctx.set_points(device_ptr=self.t_scene.data_ptr(), num_points=fr.num_points)
        own_device_budget(self.ctx)
        self.prm = _native.bp_params()
        self.groups = BP_GROUPS + G_GROUPS
        F, H, W = fr.depth.shape
        self.shape = (F, H, W)
        self.workload = (f"{shape}: ScanNet-shaped synthetic RGB-D scene, {F} frames {W}x{H}, P={fr.num_points}, "
                         f"S1-S6")

    def step(self):
        # a new scene's points (mc_scene_set_points): its ball-query grid is built inside the step
        self.ctx.set_points(device_ptr=self.t_scene.data_ptr(), num_points=self.fr.num_points)
        self.ctx.backproject(None, None, None, None, self.prm, shape=self.shape,
                             device_ptrs=(self.t_depth.data_ptr(), self.t_seg.data_ptr(), self.t_K.data_ptr(),
                                          self.t_T.data_ptr()))
        self.ctx.use_backprojection()
        self.run.step(**self.cfg)

    def work(self):
        F, H, W = self.shape
        col, lab, off, pts = self.ctx.bp_masks()
        w = graph_work(self.ctx, pts, self.fr.num_points, F)
        w.update(bp_work(self.ctx, F, H, W))
        return w

    def cpu_baseline(self):
        """the S1 port on a sample of frames spread over the scene (all threads and one thread,
        scaled per frame) + the S2-S6 port on the full mask set (identical to the device's by the
        parity tests, tests/test_gpu_bench_configs.py)."""
        fr = self.fr
        at = lambda i: (fr.depth[i].cpu().numpy(), fr.seg[i].cpu().numpy(), fr.intrinsics[i], fr.poses[i])  # noqa: E731
        s1 = s1_cpu_rate(fr.scene_points.astype(np.float32), at, fr.num_frames)
        col, lab, off, pts = self.ctx.bp_masks()
        return e2e_cpu_baseline(s1, fr.num_points, fr.num_frames, col, lab, off, pts, self.cfg)


class ShardedGraphStep(GraphStep):
    """--variant g --shard frames: ONE scene per step for the whole job (strong scaling).  Rank r
    holds its frame slice's masks (the S1 output of its frames) in HBM; a step all-gathers them
    and runs the row-block sharded S2-S6 (maskclustering_amd/frame_shard.py, graph_shard.py,
    SURVEY.md §8(e))."""

    def __init__(self, shape, seed, local):
        import torch
        from maskclustering_amd.frame_shard import FrameShardedScene
        from maskclustering_amd.pipeline import GraphRun
        from maskclustering_amd.synthetic import SHAPES, make_shape
        self.scene = s = make_shape(shape, seed=seed)
        self.dataset, self.cfg = shape_thresholds(shape)
        self.run = GraphRun(local)
        self.run.ctx.set_stream(torch.cuda.current_stream().cuda_stream)
        self.sh = FrameShardedScene(self.run, s.num_points, s.num_frames)
        lo, hi = self.sh.lo, self.sh.hi
        sel = np.nonzero((s.mask_col >= lo) & (s.mask_col < hi))[0]
        off = np.zeros(len(sel) + 1, np.int64)
        np.cumsum(np.diff(s.mask_off)[sel], out=off[1:])
        pts = np.concatenate([s.mask_points(g) for g in sel]) if len(sel) else np.zeros(0, np.int32)
        self.local = (s.mask_col[sel] - lo, s.mask_label[sel], off,
                      torch.from_numpy(pts.astype(np.int32)).to(torch.device("cuda", local)))
        self.groups = G_GROUPS
        sh = SHAPES[shape]
        self.workload = (f"{shape}: synthetic scene (SURVEY App. C), P={sh['num_points']} F={sh['num_frames']}, "
                         f"S2-S6, frames sharded over {self.sh.world} GPU(s)")

    def step(self):
        self.sh.set_local_masks(*self.local)
        self.sh.step(**self.cfg)

    def work(self):
        s = self.scene
        return graph_work(self.run.ctx, self.sh.pts.cpu().numpy(), s.num_points, s.num_frames)


class ShardedEndToEndStep(EndToEndStep):
    """--variant e2e --shard frames: ONE scene per step for the whole job (strong scaling).  Rank
    r renders and holds only its frame slice in HBM, back-projects it (S1 is independent per
    frame), the mask lists are all-gathered over RCCL and S2-S6 run row-block sharded
    (maskclustering_amd/frame_shard.py, graph_shard.py)."""

    def __init__(self, shape, seed, local):
        import torch
        import torch.distributed as dist
        from maskclustering_amd import _native
        from maskclustering_amd.frame_shard import (FrameShardedScene, balanced_frame_slices, frame_costs,
                                                    frame_slice, gather_frame_costs)
        from maskclustering_amd.pipeline import GraphRun
        from maskclustering_amd.synthetic_frames import FRAME_SHAPES, make_frames_shape
        t0 = time.perf_counter()
        F = FRAME_SHAPES[shape]["num_frames"]
        world = dist.get_world_size() if dist.is_initialized() else 1
        rank = dist.get_rank() if dist.is_initialized() else 0
        lo, hi = frame_slice(F, world, rank)
        dev = torch.device("cuda", local)
        fr = make_frames_shape(shape, seed=seed, device=f"cuda:{local}", frames=range(lo, hi), out="torch")
        costs = None
        if world > 1:  # cost-balanced slices: every rank costs its equal-count slice, then re-renders
            costs = gather_frame_costs(frame_costs(fr.depth, fr.seg, fr.intrinsics), F)
            blo, bhi = balanced_frame_slices(costs, world)[rank]
            if (blo, bhi) != (lo, hi):
                del fr
                lo, hi = blo, bhi
                fr = make_frames_shape(shape, seed=seed, device=f"cuda:{local}", frames=range(lo, hi), out="torch")
        self.fr = fr
        self.dataset, self.cfg = shape_thresholds(shape)
        self.run = GraphRun(local)
        self.ctx = self.run.ctx
        self.ctx.set_stream(torch.cuda.current_stream().cuda_stream)
        self.t_scene = torch.tensor(fr.scene_points, dtype=torch.float32, device=dev)
        self.ctx.set_points(device_ptr=self.t_scene.data_ptr(), num_points=fr.num_points)
        # one device per rank; the one-GPU rehearsal (MC_BENCH_DEVICE) splits it between the ranks
        own_device_budget(self.ctx, 0.65 / (world if os.environ.get("MC_BENCH_DEVICE") is not None else 1))
        # MC_BENCH_NATIVE_COMM=1: the sharded graph stages exchange over the library's own RCCL
        # communicator (mc_ctx_comm_init) instead of torch.distributed between calls
        native = os.environ.get("MC_BENCH_NATIVE_COMM", "0") == "1" and world > 1
        # scene-owner graph stages (default with the pipeline at N > 1; MC_BENCH_SCENE_OWNER=0: the
        # row-block sharded ones): every rank back-projects its slice of every scene, scene k's masks go
        # to rank k mod N alone, which runs S2-S6 for it (frame_shard.ScenePipeline)
        pipelined = os.environ.get("MC_BENCH_PIPELINE", "1") != "0"
        self.scene_owner = pipelined and world > 1 and os.environ.get("MC_BENCH_SCENE_OWNER", "1") != "0"
        self.sh = FrameShardedScene(self.run, fr.num_points, F, costs=costs, native_comm=native,
                                    shard_graph=not self.scene_owner)
        self.costs, self.native, self.local_dev = costs, native, local
        self._lat = None
        assert (self.sh.lo, self.sh.hi) == (lo, hi)
        up = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a)).to(dev, dt)  # noqa: E731
        self.t_depth, self.t_seg = fr.depth, fr.seg
        self.t_K = up(fr.intrinsics, torch.float64)
        self.t_T = up(fr.poses.reshape(-1, 16), torch.float64)
        self.prm = _native.bp_params()
        self.groups = BP_GROUPS + G_GROUPS
        _, H, W = fr.depth.shape
        self.F_total = F
        self.shape = (hi - lo, H, W)
        # the scene pipeline (default; MC_BENCH_PIPELINE=0 turns it off): S1 on its own context
        # and stream in a producer thread, S1 of scene k + 1 under the graph stages of scene k
        # (maskclustering_amd.frame_shard.ScenePipeline); each step is still one whole scene, and
        # the K timed steps process K whole scenes inside the timed region
        self.pipe = None
        self.timing_ctxs = [self.ctx]
        self.s1ctx = self.ctx
        if pipelined:
            from maskclustering_amd.frame_shard import ScenePipeline
            # S1 producers (contexts; MC_BENCH_S1_PRODUCERS, default one): with two, one scene's S1 kernel
            # tails are filled by the next scene's; measured +3 % for one rank's share at N = 8 but 2.2x
            # slower for whole C3 scenes on one GPU, so not the default
            nprod = int(os.environ.get("MC_BENCH_S1_PRODUCERS", "1"))
            s1ctxs = []
            for _ in range(max(1, nprod)):
                c = _native.Context(local)
                c.set_points(device_ptr=self.t_scene.data_ptr(), num_points=fr.num_points)
                own_device_budget(c, 0.6 / max(1, nprod) /
                                  (world if os.environ.get("MC_BENCH_DEVICE") is not None else 1))
                s1ctxs.append(c)
            self.s1ctx = s1ctxs[0]
            self.pipe = ScenePipeline(self.sh, s1ctxs if len(s1ctxs) > 1 else self.s1ctx, self.t_depth, self.t_seg,
                                      self.t_K, self.t_T, self.prm, scene_owner=self.scene_owner,
                                      scene_points=self.t_scene)
            self.timing_ctxs = [self.ctx] + s1ctxs
            self.pipe.warm()  # the other producers' first calls, outside the timed region
        log(f"rank {self.sh.rank}: frames [{lo}, {hi}) of {F} rendered in {time.perf_counter() - t0:.1f} s")
        self.workload = (f"{shape}: synthetic RGB-D scene, {F} frames {W}x{H}, P={fr.num_points}, "
                         f"S1-S6, frames sharded over {self.sh.world} GPU(s)")

    def step(self):
        # (scene-owner mode: the single scene is rank 0's, so rank 0's graph context holds the warmup's
        # result and the calibration's stage times)
        if self.pipe is not None:
            self.pipe.run(1, first_owner=0, **self.cfg)
            return
        self.ctx.set_points(device_ptr=self.t_scene.data_ptr(), num_points=self.fr.num_points)
        self.sh.backproject(self.t_depth, self.t_seg, self.t_K, self.t_T, self.prm)
        self.sh.step(**self.cfg)

    def run_steps(self, n):
        """n scenes; with the pipeline, S1 of scene k + 1 runs under the graph stages of scene k (in
        scene-owner mode scene k's graph stages run on rank k mod N only)"""
        if self.pipe is not None:
            self.pipe.run(n, first_owner=0, **self.cfg)
            return
        for _ in range(n):
            self.step()

    def latency_steps(self, n):
        """n scenes one at a time, every rank on each (the MC_BENCH_PIPELINE=0 path, strong scaling of
        one scene's latency): S1 of this rank's slice on the pipeline's S1 context, the mask
        all-gather, then S2-S6 row-block sharded over the ranks (graph_shard.ShardedGraph) on a graph
        context of its own.  Collective on every rank."""
        import torch
        from maskclustering_amd.frame_shard import FrameShardedScene
        from maskclustering_amd.pipeline import GraphRun
        if self._lat is None:
            run = GraphRun(self.local_dev)
            run.ctx.set_stream(torch.cuda.current_stream().cuda_stream)
            self._lat = FrameShardedScene(run, self.fr.num_points, self.F_total, costs=self.costs,
                                          native_comm=self.native, shard_graph=True)
            assert (self._lat.lo, self._lat.hi) == (self.sh.lo, self.sh.hi)
        for _ in range(n):
            self.s1ctx.set_points(device_ptr=self.t_scene.data_ptr(), num_points=self.fr.num_points)
            self._lat.backproject(self.t_depth, self.t_seg, self.t_K, self.t_T, self.prm, s1_ctx=self.s1ctx)
            self._lat.step(**self.cfg)
        return self._lat

    def work(self):
        F, H, W = self.shape
        pts = self.sh.pts.cpu().numpy()
        w = graph_work(self.ctx, pts, self.fr.num_points, self.F_total)
        w.update(bp_work(self.s1ctx, F, H, W))
        return w

    def cpu_baseline(self):
        """as EndToEndStep.cpu_baseline (rank 0 at N=1 holds every frame)"""
        fr = self.fr
        at = lambda i: (fr.depth[i].cpu().numpy(), fr.seg[i].cpu().numpy(), fr.intrinsics[i], fr.poses[i])  # noqa: E731
        s1 = s1_cpu_rate(fr.scene_points.astype(np.float32), at, len(fr.depth))
        col, lab, off = self.sh.mask_index
        return e2e_cpu_baseline(s1, fr.num_points, self.F_total, col, lab, off, self.sh.pts.cpu().numpy(),
                                self.cfg)


def c2_record(local, steps, warmup):
    """The ScanNet-sized scene (BASELINE configs[1], the north_star's "ScanNet-sized scene on 1 MI355X")
    timed in the same process with the same discipline as the main line (warmup steps, then `steps`
    steps between two device synchronisations): C2 E2E (S1-S6 from RGB-D frames resident in HBM) and
    C2 G (S2-S6 from per-frame mask sets resident in HBM).  Beside them the ports on the host: S1 on
    every frame of the scene with all threads (no sampling) + S2-S6, and one thread (S1 on 16 frames
    spread over the scene, scaled); the S1 port's output is compared with the device's (bit_exact)."""
    import torch
    from oracle import oracle
    rec = {}
    e2e = EndToEndStep("c2", 0, local)
    g = GraphStep("c2", 0, local)
    for name, r in (("c2_e2e", e2e), ("c2_g", g)):
        for _ in range(max(warmup, 1)):
            r.step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            r.step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        ctx = r.run.ctx
        ci = ctx.cluster_info()
        pairs = int(np.sum(ctx.level_sizes(ci.num_iterations)[:-1].astype(np.int64) ** 2))
        rec[name] = {"scene_ms": round(dt * 1e3, 4), "value": round(pairs / dt, 1), "unit": "mask-pairs/s",
                     "workload": r.workload + f" M={ctx.graph_info().num_masks}", "pairs_per_scene": pairs}
    fr = e2e.fr
    F, P = fr.num_frames, fr.num_points
    scene = fr.scene_points.astype(np.float32)
    depth, seg = fr.depth.cpu().numpy(), fr.seg.cpu().numpy()
    thr = oracle.default_threads()
    t0 = time.perf_counter()
    res = oracle.s1_frames(scene, depth, seg, fr.intrinsics, fr.poses, threads=thr)
    s1_all = time.perf_counter() - t0
    one = np.unique(np.linspace(0, F - 1, 16).round().astype(np.int64))
    t0 = time.perf_counter()
    oracle.s1_frames(scene, depth[one], seg[one], fr.intrinsics[one], fr.poses[one], threads=1)
    s1_one = (time.perf_counter() - t0) / len(one) * F
    col = np.concatenate([np.full(len(r[0]), c, np.int32) for c, r in enumerate(res)])
    lab = np.concatenate([r[0] for r in res]).astype(np.int32)
    off = np.concatenate([[0], np.cumsum(np.concatenate([np.diff(r[1]) for r in res]))]).astype(np.int64)
    pts = np.concatenate([r[2] for r in res]).astype(np.int32)
    dcol, dlab, doff, dpts = e2e.ctx.bp_masks()
    exact = bool(np.array_equal(col, dcol) and np.array_equal(lab, dlab) and np.array_equal(off, doff)
                 and np.array_equal(pts, dpts))
    g_all, tm = graph_cpu(P, F, col, lab, off, pts, thr, dense=True)
    g_one, _ = graph_cpu(P, F, col, lab, off, pts, 1, dense=True)
    cpu_all, cpu_one = s1_all + g_all, s1_one + g_one
    rec["c2_e2e"]["cpu_baseline"] = {
        "kind": "port", "cores": thr, "scene_ms": round(cpu_all * 1e3, 1),
        "sample": f"the whole scene: S1 port on all {F} frames ({s1_all:.2f} s, OpenMP over frames) + the dense "
                  f"S2-S6 port ({g_all:.2f} s), {thr} threads",
        "single_thread_scene_ms": round(cpu_one * 1e3, 1),
        "single_thread_sample": f"S1 port on 16 of the {F} frames scaled ({s1_one:.1f} s) + the S2-S6 port ({g_one:.2f} s)",
        "s1_bit_exact_vs_device": exact}
    rec["c2_e2e"]["speedup_vs_cpu_all_cores"] = round(cpu_all * 1e3 / rec["c2_e2e"]["scene_ms"], 1)
    rec["c2_e2e"]["speedup_vs_cpu_one_thread"] = round(cpu_one * 1e3 / rec["c2_e2e"]["scene_ms"], 1)
    rec["c2_g"]["cpu_baseline"] = {"kind": "port", "cores": thr, "scene_ms": round(g_all * 1e3, 1),
                                   "single_thread_scene_ms": round(g_one * 1e3, 1),
                                   "sample": "the dense S2-S6 port on the same masks (the e2e scene's)"}
    rec["c2_g"]["speedup_vs_cpu_all_cores"] = round(g_all * 1e3 / rec["c2_g"]["scene_ms"], 1)
    ratio_path = os.path.join(REPO, "profiles", "cpu_ratio_c2.json")
    if os.path.exists(ratio_path):  # the reference's own S2-S6, timed in the build container
        r = json.load(open(ratio_path))
        rec["c2_g"]["reference_s2_s6_s_container"] = r["reference_s"]
        rec["c2_g"]["speedup_vs_reference_s2_s6"] = round(r["reference_s"] * 1e3 / rec["c2_g"]["scene_ms"], 1)
    return rec


class PinholeIntrinsic:  # the accessors of open3d.camera.PinholeCameraIntrinsic the path reads
    def __init__(self, fx, fy, cx, cy):
        self.f, self.c = (fx, fy), (cx, cy)

    def get_focal_length(self):
        return self.f

    def get_principal_point(self):
        return self.c


class FrameDataset:  # dataset/scannet.py:34-73 over arrays
    def __init__(self, fr, frame_ids, raw_depth=True):
        self.fr, self.col = fr, {f: c for c, f in enumerate(frame_ids)}
        self.depth_scale = float(fr.meta.get("depth_scale", 1000.0))  # dataset/scannet.py:21, matterport.py:23
        for x in (fr.depth, fr.seg, fr.poses):
            x.flags.writeable = False
        if raw_depth:
            # the depth PNGs' uint16 values (the synthetic depth is quantised to millimetres), served
            # by the optional get_depth_raw hook (construction._raw_depth_scale); checked to decode
            # to exactly the float32 frames get_depth returns
            u16 = getattr(fr, "_depth_u16", None)
            if u16 is None:
                u16 = np.rint(fr.depth.astype(np.float64) * self.depth_scale).astype(np.uint16)
                if not np.array_equal((u16 / self.depth_scale).astype(np.float32).view(np.uint32),
                                      fr.depth.view(np.uint32)):
                    raise ValueError("synthetic depth is not uint16 / depth_scale")
                u16.flags.writeable = False
                fr._depth_u16 = u16
            self.get_depth_raw = lambda f: u16[self.col[f]]

    def get_intrinsics(self, f):
        return PinholeIntrinsic(*self.fr.intrinsics[self.col[f]])

    # decoded frames served from memory as read-only views (a dataset with its frames cached; the
    # reference's ScanNetDataset decodes files here, dataset/scannet.py:48-64)
    def get_extrinsic(self, f):
        return self.fr.poses[self.col[f]]

    def get_depth(self, f):
        return self.fr.depth[self.col[f]]

    def get_segmentation(self, f, align_with_depth=False):
        return self.fr.seg[self.col[f]]


def api_timing(shape, seed, steps, warmup, replay=None, with_pp=False, profile=False, fr=None, raw_depth=True):
    """The reference-API boundary exactly as main.py:17-21 calls it, on the synthetic RGB-D scene
    whose dataset object serves decoded frames from host memory (dataset/scannet.py: get_depth /
    get_segmentation / get_intrinsics / get_extrinsic): one step = mask_graph_construction +
    iterative_clustering (replay=None: the default, the reference's container orders; False:
    canonical) (+ post_process's compute, without the file export).  Wall time of that Python call
    sequence, host packing and PCIe included, per part.  raw_depth: the dataset also offers
    get_depth_raw (uint16 frames, decoded on the device); False: float32 get_depth only.
    Returns (record, frames)."""
    import cProfile
    import pstats

    import torch
    from maskclustering_amd.graph import construction, iterative_clustering
    from maskclustering_amd.synthetic_frames import make_frames_shape
    from maskclustering_amd.utils import post_process as pp

    if fr is None:
        t0 = time.perf_counter()
        fr = make_frames_shape(shape, seed=seed, device="cuda:0")
        log(f"frames {fr.depth.shape} P={fr.num_points} rendered in {time.perf_counter() - t0:.1f} s")
    fids = [int(x) for x in np.arange(0, 10 * fr.num_frames, 10)]
    args = SimpleNamespace(debug=False, **DATASET_THRESHOLDS[shape_thresholds(shape)[0]])
    ds = FrameDataset(fr, fids, raw_depth=raw_depth)
    parts = {"graph": [], "cluster": [], "post_process": []}

    def step():
        t = time.perf_counter()
        nodes, thr, mpc, pfm = construction.mask_graph_construction(args, fr.scene_points, fids, ds)
        t1 = time.perf_counter()
        objects = iterative_clustering.iterative_clustering(nodes, thr, args.view_consensus_threshold, False,
                                                            replay=replay)
        t2 = time.perf_counter()
        out = pp.post_process_objects(objects, mpc, fr.scene_points, pfm, fids, args.point_filter_threshold) \
            if with_pp else None
        t3 = time.perf_counter()
        parts["graph"].append(t1 - t)
        parts["cluster"].append(t2 - t1)
        parts["post_process"].append(t3 - t2)
        return nodes, objects, out

    for _ in range(max(warmup, 1)):
        nodes, objects, _ = step()
    for v in parts.values():
        v.clear()
    torch.cuda.synchronize()
    walls = []
    for _ in range(steps):
        t = time.perf_counter()
        step()
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t)
    if profile:
        pr = cProfile.Profile()
        pr.enable()
        step()
        pr.disable()
        pstats.Stats(pr, stream=sys.stderr).sort_stats("cumulative").print_stats(30)
    ms = 1e3 * float(np.mean(walls))
    mode = "reference" if replay is None or replay else "canonical"
    rec = {"scene_ms": round(ms, 3), "set_order": mode, "with_post_process": bool(with_pp),
           "depth_frames": "uint16 (get_depth_raw, decoded on the device)" if raw_depth else "float32 (get_depth)",
           "part_ms": {k: round(1e3 * float(np.mean(v)), 3) for k, v in parts.items() if v and (k != "post_process"
                                                                                              or with_pp)},
           "workload": f"{shape}: synthetic RGB-D scene, {fr.num_frames} frames {fr.depth.shape[2]}x{fr.depth.shape[1]}, "
                       f"P={fr.num_points}, {len(nodes)} nodes -> {len(objects)} objects; frames served from host "
                       f"memory by the dataset (PCIe and host packing in the time)"}
    return rec, fr


def run_api(a):
    """--variant api: the reference-API call sequence (api_timing) as its own line; ms_per_step is the
    wall time of main.py:17-21's calls, host packing and PCIe included (the device part is the
    e2e variant's S1-S6)."""
    rec, _ = api_timing(a.shape, a.seed, a.steps, a.warmup, replay=False if a.canonical else None,
                        with_pp=a.with_pp, profile=a.profile, raw_depth=not a.f32_depth)
    ms = rec["scene_ms"]
    res = {"metric": "reference-API graph path ms per scene (main.py:17-21 through the drop-in modules)",
           "value": ms, "unit": "ms", "n_gpus": 1, "steps": a.steps, "warmup": a.warmup,
           "ms_per_step": ms, "higher_is_better": False, "scaling": "weak", "vs_baseline": None,
           "dtype": "int32", "data": "synthetic",
           "config": {"workload": rec["workload"], "variant": "api", "set_order": rec["set_order"],
                      "with_post_process": rec["with_post_process"], "part_ms": rec["part_ms"]}}
    print(json.dumps(res), flush=True)


def run_post_process(a):
    """--variant pp: the post-processing row on the c2 RGB-D scene.  The
    drop-in graph path (S1-S6) makes the scene's objects once; each step is one drop-in
    post_process_objects call over them (utils/post_process.py:180-194: host packing, mc_pp_run,
    host lists).  cpu_baseline: oracle/pp_oracle.py (1 thread) on a bounded sample of nodes, the
    GPU run on the same sample checked bit for bit against it."""
    import torch
    from maskclustering_amd import _device
    from maskclustering_amd.graph import construction, iterative_clustering
    from maskclustering_amd.synthetic_frames import make_frames_shape
    from maskclustering_amd.utils import post_process as pp

    t0 = time.perf_counter()
    fr = make_frames_shape(a.shape, seed=0, device="cuda:0")
    fids = [int(x) for x in np.arange(0, 10 * fr.num_frames, 10)]
    log(f"frames {fr.depth.shape} P={fr.num_points} rendered in {time.perf_counter() - t0:.1f} s")
    args = SimpleNamespace(debug=False, **DATASET_THRESHOLDS[shape_thresholds(a.shape)[0]])
    t0 = time.perf_counter()
    nodes, thr, mpc, pfm = construction.mask_graph_construction(args, fr.scene_points, fids, FrameDataset(fr, fids))
    objects = iterative_clustering.iterative_clustering(nodes, thr, args.view_consensus_threshold, False)
    log(f"graph path: {len(nodes)} nodes -> {len(objects)} objects in {time.perf_counter() - t0:.1f} s")
    pfm = np.asarray(pfm)
    ctx = _device.context()
    run = lambda nl: pp.post_process_objects(nl, mpc, fr.scene_points, pfm, fids, args.point_filter_threshold)
    for _ in range(max(a.warmup, 1)):
        run(objects)
    groups = ("pp_dbscan", "pp_filter", "pp_merge")
    ctx.set_timing(True)
    ctx.reset_kernel_times()
    walls = []
    for _ in range(a.steps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        pts, masks = run(objects)
        walls.append(time.perf_counter() - t)
    kern = {g: ctx.kernel_time(g)[0] / max(ctx.kernel_time(g)[1], 1) for g in groups}
    ctx.set_timing(False)
    info = ctx.pp_info()
    kept = [o for o in objects if len(o.mask_list) >= 2]
    E = sum(len(o.point_ids) for o in kept)
    ms = 1e3 * float(np.sum(walls)) / a.steps
    res = {"metric": "post_process ms per scene (DBSCAN split + point filter + overlap merge)",
           "value": round(ms, 3), "unit": "ms", "n_gpus": 1, "steps": a.steps, "warmup": a.warmup,
           "ms_per_step": round(ms, 3), "higher_is_better": False, "scaling": "weak", "vs_baseline": None,
           "dtype": "f64", "config": {"workload": f"{a.shape}: objects of the synthetic RGB-D scene, "
                                                 f"P={fr.num_points} F={fr.num_frames}", "variant": "pp"},
           "device_ms": {g: round(v, 4) for g, v in kern.items()},
           "device_total_ms": round(sum(kern.values()), 4),
           "nodes": len(kept), "node_points": E, "dbscan_objects": info.num_objects,
           "filtered_objects": info.num_filtered, "final_objects": info.num_final,
           "output_points": int(sum(len(p) for p in pts)), "data": "synthetic"}
    budget = 15.0
    if not a.no_cpu_baseline:
        from oracle import pp_oracle
        keys = list(mpc.keys())
        kidx = {k: i for i, k in enumerate(keys)}
        col = {f: c for c, f in enumerate(fids)}
        mask_pts = [np.fromiter(mpc[k], np.int64) for k in keys]
        mask_col = np.array([col[int(k.rsplit("_", 1)[0])] for k in keys])
        sample, spent, n_pts = [], 0.0, 0
        t_cpu = 0.0
        for o in kept:                     # bounded sample, in scene order
            one = [([kidx[f"{f}_{m}"] for f, m in o.mask_list], o.visible_bool(), np.fromiter(o.point_ids, np.int64))]
            t = time.perf_counter()
            pp_oracle.post_process_objects(fr.scene_points, pfm, mask_pts, mask_col, one, args.point_filter_threshold)
            t_cpu += time.perf_counter() - t
            sample.append(o)
            n_pts += len(o.point_ids)
            if t_cpu > budget:
                break
        onodes = [([kidx[f"{f}_{m}"] for f, m in o.mask_list], o.visible_bool(), np.fromiter(o.point_ids, np.int64))
                  for o in sample]
        t = time.perf_counter()
        wp, wm = pp_oracle.post_process_objects(fr.scene_points, pfm, mask_pts, mask_col, onodes,
                                                args.point_filter_threshold)
        t_cpu_all = time.perf_counter() - t
        torch.cuda.synchronize()
        t = time.perf_counter()
        gp, gm = run(sample)
        t_gpu = time.perf_counter() - t
        same = len(gp) == len(wp) and all(np.array_equal(x, y) for x, y in zip(gp, wp)) and \
            [[(f, m, c) for f, m, c in x] for x in gm] == \
            [[(int(keys[q].rsplit("_", 1)[0]), int(keys[q].rsplit("_", 1)[1]), c) for q, c in x] for x in wm]
        res["cpu_baseline"] = {"kind": "port", "cores": 1, "sample": f"{len(sample)} of {len(kept)} nodes, "
                               f"{n_pts} of {E} node points (oracle/pp_oracle.py incl. the merge over the sample)",
                               "cpu_ms": round(1e3 * t_cpu_all, 1), "gpu_ms_same_sample": round(1e3 * t_gpu, 3),
                               "bit_exact_on_sample": bool(same)}
    print(json.dumps(res), flush=True)


def run_sweep(a):
    """--variant sweep: BASELINE configs[4], the full ScanNet val sweep, scene-parallel as the reference's
    run.py:33-50 runs it (one process per GPU, scene i on rank i mod N, no data-path collective).
    A scene = S1-S6 from its RGB-D frames resident in HBM (the e2e variant's step: set_points builds the
    scene's ball-query grid, mc_backproject, mc_graph_build + mc_cluster_run); the rank's scenes are
    cycled from a pool of --pool distinct synthetic ScanNet-shaped scenes rendered once (seeds
    seed + rank * pool + j).  value = wall time of all --scenes scenes (max over ranks)."""
    import torch
    import torch.distributed as dist
    from maskclustering_amd.sweep import SceneSweep, scenes_of
    from maskclustering_amd.synthetic_frames import make_frames_shape

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    mine = scenes_of(rank, world, a.scenes)
    pool = []
    t0 = time.perf_counter()
    for j in range(min(a.pool, max(len(mine), 1))):
        fr = make_frames_shape(a.shape, seed=a.seed + rank * a.pool + j, device=f"cuda:{local}", out="torch")
        pool.append((fr, torch.tensor(fr.scene_points, dtype=torch.float32, device=dev),
                     torch.from_numpy(np.ascontiguousarray(fr.intrinsics)).to(dev),
                     torch.from_numpy(np.ascontiguousarray(fr.poses.reshape(-1, 16))).to(dev)))
    log(f"rank {rank}: {len(mine)} scenes from a pool of {len(pool)} rendered in {time.perf_counter() - t0:.1f} s")
    sw = SceneSweep(local, shape_thresholds(a.shape)[1], stream=torch.cuda.current_stream().cuda_stream)
    objects = []

    def scene(j):
        fr, pts, K, T = pool[j % len(pool)]
        return sw.run_scene(pts, fr.depth, fr.seg, K, T)

    for j in range(min(len(pool), max(a.warmup, 1))):
        scene(j)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for j in range(len(mine)):
        objects.append(scene(j))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    wall = float(elapsed.item())
    if rank == 0:
        fr = pool[0][0]
        res = {"metric": "full-sweep end-to-end wall time (BASELINE configs[4]: 312 ScanNet val scenes, scene-parallel)",
               "value": round(wall, 3), "unit": "s", "n_gpus": world, "steps": a.scenes, "warmup": a.warmup,
               "ms_per_step": round(1e3 * wall / max(a.scenes, 1) * world, 3), "higher_is_better": False,
               "scaling": "strong", "vs_baseline": None, "dtype": "int32", "data": "synthetic",
               "config": {"workload": f"{a.scenes} scenes of {a.shape} ({fr.num_frames} frames {fr.depth.shape[2]}x"
                                      f"{fr.depth.shape[1]}, P={fr.num_points}), S1-S6 per scene, scene i on rank "
                                      f"i mod {world}, each rank cycling {len(pool)} distinct rendered scenes",
                          "variant": "sweep", "parallelism": f"scene-parallel x{world}",
                          "scenes_per_s": round(a.scenes / wall, 3),
                          "rank0_objects_per_scene": round(float(np.mean(objects)), 1) if objects else 0}}
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--variant", choices=["g", "e2e", "pp", "api", "sweep"], default="e2e")
    ap.add_argument("--scenes", type=int, default=312, help="sweep: scenes of the whole job (ScanNet val: 312)")
    ap.add_argument("--pool", type=int, default=4, help="sweep: distinct rendered scenes per rank")
    ap.add_argument("--with-pp", action="store_true", help="api: include post_process's compute")
    ap.add_argument("--profile", action="store_true", help="api: cProfile one extra step to stderr")
    ap.add_argument("--canonical", action="store_true", help="api: iterative_clustering(replay=False), contents "
                                                             "only (the default is the reference's set orders, "
                                                             "INTEGRATION.md §4)")
    ap.add_argument("--f32-depth", action="store_true", help="api: the dataset hands out float32 get_depth only "
                                                             "(default: also get_depth_raw, uint16 frames)")
    ap.add_argument("--shape", default=None, help="default: c3 (g, e2e), c2 (api, pp, sweep)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true", help="skip the C2 E2E / G record (N=1 only)")
    ap.add_argument("--no-latency", action="store_true", help="skip the one-scene-at-a-time latency record")
    ap.add_argument("--shard", choices=["scene", "frames"], default="frames",
                    help="frames: one scene, its frames split over the ranks, S2-S6 row-block sharded (strong "
                         "scaling; the north_star's ScanNet++-sized C3 by default); scene: every rank its own "
                         "scene (weak scaling, the reference's run.py sweep, BASELINE configs[4])")
    args = ap.parse_args()
    if args.shape is None:
        args.shape = "c3" if args.variant in ("g", "e2e") else "c2"
    if args.variant == "pp":
        return run_post_process(args)
    if args.variant == "api":
        return run_api(args)
    if args.variant == "sweep":
        return run_sweep(args)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knob for the multi-rank path on a one-GPU box (never for a measured run): every rank on
    # device MC_BENCH_DEVICE, collectives over gloo (host tensors) instead of RCCL
    if os.environ.get("MC_BENCH_DEVICE") is not None:
        local = int(os.environ["MC_BENCH_DEVICE"])
    torch.cuda.set_device(local)
    if world > 1:
        if os.environ.get("MC_BENCH_BACKEND", "nccl") == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    frames = args.shard == "frames"
    if frames:  # one scene, frame slices per rank (strong scaling)
        runner = (ShardedGraphStep if args.variant == "g" else ShardedEndToEndStep)(args.shape, args.seed, local)
    else:  # every rank its own scene (weak scaling)
        runner = (GraphStep if args.variant == "g" else EndToEndStep)(args.shape, args.seed + rank, local)
    ctx = runner.run.ctx
    # contexts whose group timers the line reads (the scene pipeline runs S1 on a context of its own)
    tctxs = getattr(runner, "timing_ctxs", [ctx])

    def ktime(g):  # (ms, launches) of group g from the context that ran it
        return max((c.kernel_time(g) for c in tctxs), key=lambda v: v[1])

    for _ in range(args.warmup):
        runner.step()
    torch.cuda.synchronize()
    # (scene-owner mode: the warmup and calibration scenes are rank 0's, the other ranks hold no graph
    # result; they only time their share and join the max-reduce)
    has_graph = rank == 0 or not getattr(runner, "scene_owner", False)
    pairs_per_step = 0
    if has_graph:
        ci = ctx.cluster_info()
        sizes = ctx.level_sizes(ci.num_iterations)
        pairs_per_step = int(np.sum(sizes[:-1].astype(np.int64) ** 2))

    # calibration pass with per-group event timing: find the dominant kernel group
    for c in tctxs:
        c.reset_kernel_times()
        c.set_timing(True)
    runner.step()
    for c in tctxs:
        c.synchronize()
    calib = {g: ktime(g) for g in runner.groups}
    for c in tctxs:
        c.set_timing(False)
    work = runner.work() if has_graph else {}
    for g in BP_GROUPS:  # S1 models are scene totals: per launch = total / the group's launches per scene
        if g in work and calib.get(g, (0, 0))[1]:
            b, tot, model, alt = work[g]
            work[g] = (b, tot / calib[g][1], model + " per scene / launches per scene", alt)
    dominant = max((g for g in calib if g in work), key=lambda g: calib[g][0]) if work else BP_GROUPS[0]
    log("calibration (ms):", json.dumps({k: round(v[0], 4) for k, v in calib.items()}), "dominant:", dominant)

    # timed region: barrier + synchronize on both sides; live HIP-event timing of the dominant
    # group only (one event pair per launch of the group, on the context stream)
    for c in tctxs:
        c.reset_kernel_times()
        c.set_timing_filter(dominant)
        c.set_timing(True)
    pipe = getattr(runner, "pipe", None)
    if pipe is not None:
        pipe.gather_s, pipe.gathers = 0.0, 0
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if hasattr(runner, "run_steps"):
        runner.run_steps(args.steps)
    else:
        for _ in range(args.steps):
            runner.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    for c in tctxs:
        c.set_timing(False)
    dom_ms, dom_n = ktime(dominant)
    gather_ms = 1e3 * pipe.gather_s / max(pipe.gathers, 1) if pipe is not None else 0.0
    # the one-scene-at-a-time latency beside the pipelined throughput (frame-sharded e2e with the pipeline):
    # the same barrier / synchronize discipline, max over ranks
    lat_elapsed, lat_n = 0.0, 0
    if pipe is not None and hasattr(runner, "latency_steps") and not args.no_latency:
        lat_n = max(2, min(args.steps, 5))
        runner.latency_steps(1)  # its graph context's first call
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        tl = time.perf_counter()
        runner.latency_steps(lat_n)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        lat_elapsed = time.perf_counter() - tl
    from maskclustering_amd.frame_shard import rccl_comm_ranks
    rccl_ranks = rccl_comm_ranks() if world > 1 else None
    t = torch.tensor([elapsed, gather_ms, lat_elapsed], dtype=torch.float64,
                     device="cuda" if world == 1 or dist.get_backend() == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, gather_ms, lat_elapsed = (float(x) for x in t.tolist())
    if not has_graph:
        dist.destroy_process_group()
        return

    gi = ctx.graph_info()
    s6_ms = sum(calib.get(g, (0.0, 0))[0] for g in ("s6_columns", "s6_pairs", "s6_components", "s6_merge"))
    total_pairs = pairs_per_step * args.steps * (1 if frames else world)
    value = total_pairs / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    # HBM bytes per launch of every kernel group from the committed rocprofv3 PMC passes of the
    # same workload (scripts/pmc_summary.py; FETCH_SIZE doubled per the gfx950 note in
    # MI355X_MICROARCH.md)
    pmc_path = os.path.join(REPO, "profiles", f"pmc_traffic_{args.variant}_{args.shape}.json")
    pmc = json.load(open(pmc_path)).get("groups", {}) if os.path.exists(pmc_path) else {}
    roof = roofline_entry(work[dominant], (dom_ms / max(dom_n, 1)) / 1e3, pmc.get(dominant))
    roof["kernel"] = dominant
    roof["launches_timed"] = int(dom_n)
    if dominant == "bp_denoise":
        s1c = getattr(runner, "s1ctx", None) or getattr(runner, "ctx", None)
        nvox = int(s1c.bp_candidates()[:, 3].sum()) if s1c is not None else None
        roof["valu"] = denoise_valu(runner.shape[0], calib[dominant][1], dom_ms / max(dom_n, 1) / 1e3, nvox)
    if pmc.get(dominant):
        roof["traffic_source"] = os.path.relpath(pmc_path, REPO)
    stages = {}
    for g, (ms, n) in calib.items():
        if g in work and n:
            e = roofline_entry(work[g], ms / n / 1e3, pmc.get(g))
            stages[g] = {k: e[k] for k in ("bound", "achieved", "unit", "frac", "avg_launch_ms", "model")
                         if k in e}
            for k in ("alt_frac", "traffic_frac_hbm"):
                if k in e:
                    stages[g][k] = e[k]
            if "dense-equivalent" in e["model"]:
                # the reference's dense work over this sparse kernel's time: a ratio, not a roofline
                # fraction (it exceeds 1); frac is then the kernel's own bytes model (alt_frac) where
                # one is defined, else absent
                stages[g]["dense_equiv_ratio"] = stages[g].pop("frac")
                if "alt_frac" in stages[g]:
                    stages[g]["frac"] = stages[g].pop("alt_frac")

    cpu = None
    ms_per_step_pre = elapsed / args.steps * 1e3
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = runner.cpu_baseline()
        ratio_path = os.path.join(REPO, "profiles", f"cpu_ratio_{args.shape}.json")
        if os.path.exists(ratio_path) and args.variant == "g":
            r = json.load(open(ratio_path))
            cpu["reference_context"] = {
                "source": os.path.relpath(ratio_path, REPO),
                "note": "the reference's own S2-S6 (imported unmodified, Appendix B harness) and this C port "
                        "on the same synthetic scene, both on the 8-core build container (scripts/cpu_ratio.py)",
                "reference_s": r["reference_s"], "port_s_container": r["port_s"],
                "port_threads_container": r["port_threads"], "reference_over_port": r["reference_over_port"]}
        elif args.variant == "e2e":
            cpu["reference_context"] = {
                "note": "the reference's own S1 (utils/mask_backprojection.py) calls Open3D and pytorch3d, which are not "
                        "installed in the build container or on the box, so only its S2-S6 was timed against the C port "
                        f"(profiles/cpu_ratio_c2.json: the reference over the port for S2-S6 on C2); S1 here is the "
                        "port's restatement (oracle/s1_oracle.c), timed on all host threads (value) and on one (single_thread)"}
        fit_path = os.path.join(REPO, "profiles", "cpu_ref_fit.json")
        if os.path.exists(fit_path) and args.variant in ("e2e", "g"):
            # the reference's S2-S6 at this scene's M, EXTRAPOLATED from its T(M) fit over C1 / C2 / 2xC2 (it
            # cannot run C3 / C4: dense M x M float32 matrices)
            fit = json.load(open(fit_path))
            M_run = int(ctx.graph_info().num_masks)
            t_ref = fit["a"] * M_run ** fit["b"]
            cpu.setdefault("reference_context", {})["reference_s2_s6_extrapolated"] = {
                "seconds": round(t_ref, 1), "M": M_run, "fit": f"T(M) = {fit['a']:.4g} * M^{fit['b']}",
                "points": [(p["shape"], p["M"], p["reference_s"]) for p in fit["points"]],
                "label": "EXTRAPOLATED (not run): the reference's own S2-S6 timed on the 8-core build container at "
                         "C1, C2 and 2xC2 under configs/scannet.json thresholds (scripts/cpu_ratio.py, "
                         "scripts/cpu_ref_fit.py); S1 excluded (Open3D / pytorch3d absent)",
                "source": os.path.relpath(fit_path, REPO),
                "over_device_scene": round(t_ref * 1e3 / max(ms_per_step_pre, 1e-9), 1)}

    if cpu and cpu.get("s1_crop_candidates_per_frame") and stages.get("bp_query"):
        # SURVEY.md §8(d)'s S1 bytes count each mask's cropped candidates (12·c̄ per mask): the reference's
        # crop (every scene point inside the mask's AABB) is never made on the device, so c̄ comes from
        # the port's crop (oracle/s1_oracle.c, stats "ncand") on the cpu_baseline's sampled frames, scaled
        # to the scene's frames; the query kernel reads only the 2r cells around each mask point
        q = stages["bp_query"]
        n_q = calib["bp_query"][1]  # launches per scene (the calibration step is one scene)
        cand_b = 12.0 * cpu["s1_crop_candidates_per_frame"] * runner.shape[0] / max(n_q, 1)
        with_c = work["bp_query"][1] + cand_b
        avg_q = q["avg_launch_ms"] / 1e3
        q["survey_model"] = "12·Σ mask points + 4·Σ neighbour ids + 12·Σ cropped candidates (c̄ sampled, see note)"
        q["survey_frac"] = round(with_c / avg_q / 1e9 / HBM_PEAK_GBS, 4)
        if pmc.get("bp_query"):
            q["traffic_over_survey_model"] = round(float(pmc["bp_query"]["bytes_per_launch"]) / with_c, 2)
        q["survey_note"] = (f"c̄: {cpu['s1_crop_candidates_per_frame']:.0f} cropped scene points per frame (summed over its "
                            "masks) in the S1 port's crop on the cpu_baseline frames, scaled to the scene")

    secondary = None
    if rank == 0 and world == 1 and not args.no_secondary and args.variant in ("e2e", "g"):
        secondary = c2_record(local, max(3, min(args.steps, 10)), args.warmup)
        # the boundary main.py calls (reference-API drop-ins, frames from host memory) on the same C2
        # scene: default (the reference's container orders) with post_process, and canonical
        n_api = max(3, min(args.steps, 5))
        api, fr_c2 = api_timing("c2", 0, n_api, 2, replay=None, with_pp=True)
        can, _ = api_timing("c2", 0, n_api, 2, replay=False, fr=fr_c2)
        f32, _ = api_timing("c2", 0, n_api, 2, replay=None, fr=fr_c2, raw_depth=False)
        e2e_ms = secondary["c2_e2e"]["scene_ms"]
        api["over_device_e2e"] = round((api["scene_ms"] - api["part_ms"].get("post_process", 0.0)) / e2e_ms, 2)
        can["over_device_e2e"] = round(can["scene_ms"] / e2e_ms, 2)
        f32["over_device_e2e"] = round(f32["scene_ms"] / e2e_ms, 2)
        secondary["c2_api"] = api
        secondary["c2_api_canonical"] = can
        secondary["c2_api_f32_depth"] = f32
        secondary["c2_pp"] = {"scene_ms": api["part_ms"].get("post_process"),
                              "note": "post_process_objects (utils/post_process.py:180-194: DBSCAN split, point "
                                      "filter, overlap merge; host packing included) on the c2_api run's objects"}

    if rank == 0:
        line = {
            "metric": "mask-pair consensus counts/sec (per-scene graph build+cluster)",
            "value": round(value, 1),
            "unit": "mask-pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "strong" if frames else "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic",
            "config": {"workload": runner.workload + f" M={gi.num_masks}", "variant": args.variant,
                       "dataset_config": f"configs/{runner.dataset}.json", "thresholds": runner.cfg,
                       "scene_ms": round(ms_per_step, 4), "pairs_per_scene": pairs_per_step,
                       "iterations": int(ci.num_iterations), "objects": int(ci.num_objects),
                       "stage_ms": {k: round(v[0], 4) for k, v in calib.items()},
                       "parallelism": (f"frame-sharded x{world}" + (", scene-owner graph stages"
                                                                     if getattr(runner, "scene_owner", False) else "")
                                       if frames else f"scene-parallel x{world}"),
                       "scene_pipeline": getattr(runner, "pipe", None) is not None,
                       "s1_producers": len(runner.pipe.s1s) if getattr(runner, "pipe", None) is not None else 0},
            # SURVEY.md §8(d)'s own definition of the pair metric: the same pairs over S6's time only
            "pairs_per_s_s6": round(pairs_per_step / max(s6_ms / 1e3, 1e-12), 1),
            "pairs_per_s_s6_def": "sum_t N_t^2 / sum_t (S6 iteration t's device time: s6_columns + s6_pairs + "
                                  "s6_components + s6_merge of the calibration step, HIP events)",
            "roofline": roof,
            "stage_roofline": stages,
            "cpu_baseline": cpu,
        }
        if world > 1:
            line["rccl_comm_ranks"] = rccl_ranks  # ncclCommCount on the job's communicator (None under gloo)
            line["backend"] = dist.get_backend()
        if pipe is not None:
            line["gather_ms_per_scene"] = round(gather_ms, 4)
            line["gather_note"] = ("host wall time per scene in gather_masks (mask metadata all-gather + point-id "
                                   "gather to the scene's owner), max over ranks; it includes waiting for the slowest "
                                   "rank's S1 of the scene" if world > 1 else "one process: no collective")
        if lat_n:
            line["latency"] = {
                "ms_per_scene": round(1e3 * lat_elapsed / lat_n, 4), "scenes": lat_n,
                "mode": "one scene at a time, every rank on it (MC_BENCH_PIPELINE=0 path): S1 of each rank's "
                        "frame slice, mask all-gather, S2-S6 row-block sharded over the ranks; max over ranks",
                "scene_ms_pipelined": round(ms_per_step, 4)}
        if secondary:
            line["secondary"] = secondary
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
