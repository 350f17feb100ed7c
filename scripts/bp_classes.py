"""Diagnostic: slot counts per denoise size class on a bench-shaped scene (run under
rocprofv3 --kernel-trace for the per-class kernel durations).

    python scripts/bp_classes.py [shape]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from maskclustering_amd import _native  # noqa: E402
from maskclustering_amd.synthetic_frames import make_frames_shape  # noqa: E402

shape = sys.argv[1] if len(sys.argv) > 1 else "c2"
fr = make_frames_shape(shape, seed=0, device="cuda")
ctx = _native.Context(0)
ctx.set_points(fr.scene_points.astype(np.float32))
for rep in range(2):
    ctx.backproject(fr.depth, fr.seg, fr.intrinsics, fr.poses)
    ctx.synchronize()
st = ctx.bp_candidates()
nv = st[:, 3]
edges = [0, 512, 1024, 2048, 3072, 1 << 30]
for k in range(5):
    sel = (nv > edges[k]) & (nv <= edges[k + 1])
    print(f"class {k} (<= {edges[k + 1]}): slots {int(sel.sum())} voxels {int(nv[sel].sum())}")
print("frames", fr.num_frames, "slots", len(nv))
