"""Benchmark of the view-consensus graph path on MI355X.

A step = one pass of the hot path over one synthetic ScanNet-shaped scene
(BASELINE.json configs[1]: ~250 frames, ~240k points, ~15k masks): graph
construction S2–S5 (point lists, boundary, containment, under-segmentation,
observer thresholds), iterative clustering S6 (all thresholds) and the final
per-object point sets — from per-frame mask sets resident in HBM to final
components + merged bitsets in HBM.

metric: mask-pair consensus counts/sec = Σ_t N_t² (the ordered node pairs whose
view consensus the reference evaluates, graph/iterative_clustering.py:20-29)
summed over the scenes of all ranks ÷ max-over-ranks wall time of the steps.
ms_per_step is the per-scene graph build + cluster time (BASELINE.json's
first metric).  Multi-GPU: one process per GPU, each rank its own scene
(scene-parallel, the reference's run.py:33-50 pattern): weak scaling, no
data-path collective.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--shape c2] [--no-cpu-baseline]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md)
INT8_MFMA_PEAK_TOPS = 5000.0  # dense int8 MFMA (2x the 2.5 PF bf16 dense)
CFG = dict(mask_visible_threshold=0.3, undersegment_filter_threshold=0.3, view_consensus_threshold=0.9,
           contained_threshold=0.8)  # configs/scannet.json


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def algorithmic_work(scene, run, F):
    """Per-launch algorithmic bytes / ops of every timed kernel group."""
    ctx = run.ctx
    gi = ctx.graph_info()
    P, M, nnz = scene.num_points, gi.num_masks, int(scene.mask_off[-1])
    FW = (F + 63) // 64
    deg = np.bincount(scene.mask_pts, minlength=P).astype(np.int64)
    bnd = ctx.boundary(P).astype(bool)
    pts = scene.mask_pts
    nb = ~bnd[pts]
    # S3: every mask reads its ids (4 B) + boundary flag (1 B); every non-boundary point its
    # offsets (8 B) and list entries (4 B each); writes its contained row + flags.
    s3_bytes = 8 * M + 5 * nnz + int(np.sum(8 + 4 * deg[pts[nb]])) + 4 * gi.num_contained + 5 * M
    # S2: read mask ids, write + sort point lists (r/w), offsets, boundary, point-frame bits
    s2_bytes = 4 * nnz + 2 * 4 * nnz + 2 * 4 * nnz + 8 * P + P + 8 * P * FW
    # S4: dense-equivalent observer GEMM VF·VFᵀ (construction.py:84) — 2·M²·F int8 ops
    s4_ops = 2.0 * M * M * F
    s7_bytes = 2 * 4 * nnz + 4 * int(ctx.cluster_info().num_object_points)
    return {
        "s2_point_lists": ("hbm", float(s2_bytes)),
        "s3_masks": ("hbm", float(s3_bytes)),
        "s4_observer_hist": ("mfma", s4_ops),
        "s7_points": ("hbm", float(s7_bytes)),
    }


def cpu_baseline(scene, threads):
    from oracle import oracle
    os.environ.setdefault("OMP_NUM_THREADS", str(threads))
    tm = {}
    t0 = time.perf_counter()
    oracle.run(scene.num_points, scene.num_frames, scene.mask_col, scene.mask_label, scene.mask_off,
               scene.mask_pts, timings=tm, **CFG)
    wall = time.perf_counter() - t0
    cpu_s = tm["s2"] + tm["s3"] + tm["s4"] + tm["s6"]
    return tm, wall, cpu_s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--shape", default="c2")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from maskclustering_amd.pipeline import GraphRun
    from maskclustering_amd.synthetic import SHAPES, make_shape

    scene = make_shape(args.shape, seed=args.seed + rank)  # every rank its own scene (weak scaling)
    run = GraphRun(local)
    run.ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    run.set_scene(scene)

    for _ in range(args.warmup):
        run.step(**CFG)
    torch.cuda.synchronize()
    ci = run.ctx.cluster_info()
    sizes = run.ctx.level_sizes(ci.num_iterations)
    pairs_per_step = int(np.sum(sizes[:-1].astype(np.int64) ** 2))

    # calibration pass with per-group event timing: find the dominant kernel group
    groups = ["s2_point_lists", "s3_masks", "s3_undo_s5", "s4_observer_hist", "s6_columns", "s6_pairs",
              "s6_components", "s6_merge", "s7_points"]
    run.ctx.reset_kernel_times()
    run.ctx.set_timing(True)
    run.step(**CFG)
    run.ctx.synchronize()
    calib = {g: run.ctx.kernel_time(g)[0] for g in groups}
    run.ctx.set_timing(False)
    work = algorithmic_work(scene, run, scene.num_frames)
    dominant = max((g for g in calib if g in work), key=lambda g: calib[g])
    log("calibration (ms):", json.dumps({k: round(v, 4) for k, v in calib.items()}), "dominant:", dominant)

    # timed region: barrier + synchronize on both sides; live HIP-event timing of the dominant
    # group only (one event pair per step)
    run.ctx.reset_kernel_times()
    run.ctx.set_timing_filter(dominant)
    run.ctx.set_timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run.step(**CFG)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    run.ctx.set_timing(False)
    dom_ms, dom_n = run.ctx.kernel_time(dominant)
    t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    gi = run.ctx.graph_info()
    total_pairs = pairs_per_step * args.steps * world
    value = total_pairs / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    bound, per_launch = work[dominant]
    avg_s = (dom_ms / max(dom_n, 1)) / 1e3
    if bound == "hbm":
        achieved = per_launch / avg_s / 1e9
        roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None}
    else:
        achieved = per_launch / avg_s / 1e12
        roof = {"bound": "mfma", "achieved": round(achieved, 2), "peak": INT8_MFMA_PEAK_TOPS, "unit": "TFLOP/s",
                "frac": round(achieved / INT8_MFMA_PEAK_TOPS, 4), "traffic": None}
    roof["kernel"] = dominant
    roof["avg_launch_ms"] = round(avg_s * 1e3, 5)
    roof["algorithmic_per_launch"] = per_launch
    # HBM bytes per launch of the same kernel group from the committed rocprofv3 PMC passes
    # (scripts/pmc_summary.py; FETCH_SIZE doubled per the gfx950 note in MI355X_MICROARCH.md)
    pmc_path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if bound == "hbm" and os.path.exists(pmc_path):
        g = json.load(open(pmc_path)).get("groups", {}).get(dominant)
        if g:
            roof["traffic"] = round(g["bytes_per_launch"], 0)
            roof["traffic_source"] = "profiles/pmc_traffic.json"

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = min(16, os.cpu_count() or 1)
        tm, wall, cpu_s = cpu_baseline(scene, threads)
        cpu = {"value": round(tm["pairs"] / cpu_s, 1), "unit": "mask-pairs/s", "cores": tm["threads"],
               "kind": "port",
               "sample": f"oracle/mcgraph_oracle.c S2-S6 on the same {args.shape} scene (1 full scene, "
                         f"{cpu_s:.2f} s: S2 {tm['s2']:.2f} S3 {tm['s3']:.2f} S4 {tm['s4']:.2f} S6 {tm['s6']:.2f})",
               "scene_ms": round(cpu_s * 1e3, 1)}

    if rank == 0:
        shape = SHAPES[args.shape]
        line = {
            "metric": "mask-pair consensus counts/sec (per-scene graph build+cluster)",
            "value": round(value, 1),
            "unit": "mask-pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic",
            "config": {"workload": f"{args.shape}: ScanNet-shaped synthetic scene (SURVEY App. C), "
                                   f"P={shape['num_points']} F={shape['num_frames']} M={gi.num_masks}",
                       "scene_ms": round(ms_per_step, 4), "pairs_per_scene": pairs_per_step,
                       "iterations": int(ci.num_iterations), "objects": int(ci.num_objects),
                       "parallelism": f"scene-parallel x{world}"},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
