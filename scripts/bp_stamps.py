"""Diagnostic: per-step clock shares of k_bp_denoise (library built with -DMC_BP_STAMPS,
selected with MCGRAPH_LIB) on a bench-shaped scene, plus the slot size distribution.

    MCGRAPH_LIB=maskclustering_amd/libmcgraph_stamps.so python scripts/bp_stamps.py [shape] [frames]
"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from maskclustering_amd import _native  # noqa: E402
from maskclustering_amd.synthetic_frames import make_frames_shape  # noqa: E402

shape = sys.argv[1] if len(sys.argv) > 1 else "c2"
f0 = int(sys.argv[2]) if len(sys.argv) > 2 else 0
nf = int(sys.argv[3]) if len(sys.argv) > 3 else 250
fr = make_frames_shape(shape, seed=0, device="cuda", frames=range(f0, f0 + nf))
ctx = _native.Context(0)
L = _native.load()
L.mc_debug_bp_stamps.restype = ctypes.c_int
L.mc_debug_bp_stamps.argtypes = [ctypes.c_void_p]
ctx.set_points(fr.scene_points.astype(np.float32))
buf = np.zeros(48, np.uint64)
for rep in range(3):
    L.mc_debug_bp_stamps(buf.ctypes.data)
    ctx.set_timing(True)
    ctx.reset_kernel_times()
    t0 = time.perf_counter()
    ctx.backproject(fr.depth, fr.seg, fr.intrinsics, fr.poses)
    ctx.synchronize()
    dt = time.perf_counter() - t0
    L.mc_debug_bp_stamps(buf.ctypes.data)
    groups = {g: round(ctx.kernel_time(g)[0], 3) for g in ("bp_pixels", "bp_voxel", "bp_denoise", "bp_query")}
names = ["slot-top", "bbox", "cells", "bucket-scan", "scatter", "ncount", "union", "ranks", "labels", "filter",
         "knn", "stats", "survivors"]
print("call ms", round(dt * 1e3, 2), groups)
nslots = max(int(buf[14]), 1)
print("LDS-class slots", int(buf[14]), "mean voxels", round(float(buf[15]) / nslots, 1))
for off, kern in ((16, "k_bp_denoise_lds"), (0, "k_bp_denoise (large slots)")):
    tot = float(buf[off:off + 13].sum()) + (float(buf[34] + buf[35]) if off == 16 else 0.0)
    print(kern, "total workgroup-busy ms (100 MHz clock)", round(tot / 1e5, 2))
    for k, n in enumerate(names):
        v = float(buf[off + k]) + (float(buf[34] + buf[35]) if off == 16 and n == "knn" else 0.0)
        per = f"{v / 100.0 / nslots:8.2f} us/slot" if off == 16 else ""
        print(f"  {n:12s} {100.0 * v / max(tot, 1):6.2f} % {per}")
print("k-NN sub-phases us/slot: main list pass", round(float(buf[34]) / 100.0 / nslots, 2), "ring search",
      round(float(buf[35]) / 100.0 / nslots, 2), "whole-cloud fallback", round(float(buf[26]) / 100.0 / nslots, 2))
print("k-NN points deferred to the ring search", int(buf[30]), "(list overflow", int(buf[32]), "/ < k kept in the list",
      int(buf[33]), ")", "near-tied keys redone exactly", int(buf[31]))
print("knn points", int(buf[13]), "candidates/point", round(float(buf[29]) / max(int(buf[13]), 1), 1),
      "fallbacks", int(buf[31]))
vt = [float(buf[k]) for k in (36, 38, 40, 37, 39)]
vtot = max(sum(vt), 1.0)
print("k_bp_voxel_lds workgroup-busy shares:", {n: f"{100 * v / vtot:.1f} %" for n, v in
      zip(("0 min bound", "1a points+keys+probes", "1b masks+ids+sums", "1 exit", "2 means + slot set-up"), vt)},
      "total ms", round(vtot / 1e5, 2))
st = ctx.bp_candidates()
for c, n in ((2, "npix"), (3, "nvox"), (4, "ndbscan"), (5, "nsor")):
    v = st[:, c]
    print(n, "mean", round(float(v.mean()), 1), "p99", int(np.percentile(v, 99)), "max", int(v.max()))
