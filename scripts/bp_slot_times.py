"""Diagnostic: per-slot denoise busy time (stamps build, MCGRAPH_LIB) against slot shape,
one batch holding every frame.

    MC_BP_BATCH_PIXELS=80000000 MCGRAPH_LIB=maskclustering_amd/libmcgraph_stamps.so \\
        python scripts/bp_slot_times.py [shape] [first frame] [frames]
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from maskclustering_amd import _native  # noqa: E402
from maskclustering_amd.synthetic_frames import make_frames_shape  # noqa: E402

shape = sys.argv[1] if len(sys.argv) > 1 else "c2"
f0 = int(sys.argv[2]) if len(sys.argv) > 2 else 0
nf = int(sys.argv[3]) if len(sys.argv) > 3 else None
fr = make_frames_shape(shape, seed=0, device="cuda", **({"frames": range(f0, f0 + nf)} if nf else {}))
ctx = _native.Context(0)
L = _native.load()
L.mc_debug_bp_slot_times.argtypes = [ctypes.c_void_p, ctypes.c_int]
ctx.set_points(fr.scene_points.astype(np.float32))
for rep in range(2):
    ctx.backproject(fr.depth, fr.seg, fr.intrinsics, fr.poses)
    ctx.synchronize()
st = ctx.bp_candidates()
ns = len(st)
tm = np.zeros(1 << 16, np.uint32)
L.mc_debug_bp_slot_times(tm.ctypes.data, 1 << 16)
us = tm[:ns] / 100.0
nv, nd, nsor = st[:, 3], st[:, 4], st[:, 5]
print("slots", ns, "total busy ms", round(us.sum() / 1e3, 1))
for q in (50, 90, 99, 99.9, 100):
    print(f"  p{q}: {np.percentile(us, q):9.1f} us")
order = np.argsort(-us)
print("slowest slots: us nvox ndbscan nsor")
for i in order[:15]:
    print(f"  {us[i]:9.1f} {nv[i]:6d} {nd[i]:6d} {nsor[i]:6d}")
for lo, hi in ((0, 512), (512, 1024), (1024, 2048), (2048, 3072), (3072, 4096), (4096, 16384)):
    sel = (nv > lo) & (nv <= hi)
    if sel.any():
        print(f"class ({lo},{hi}]: n {int(sel.sum())} mean {us[sel].mean():8.1f} us  p50 {np.median(us[sel]):8.1f}"
              f"  max {us[sel].max():9.1f}  us/voxel {us[sel].sum() / nv[sel].sum():.3f}")
print("share of busy time in the slowest 1% slots:", round(float(np.sort(us)[-max(ns // 100, 1):].sum() / us.sum()), 3))
