"""Diagnostic: one mc_backproject call on a golden S1 case with MC_BP_DEBUG_SYNC=1 (every S1
group synchronised and reported on stderr), to locate a stalled group.

    MC_BP_DEBUG_SYNC=1 python scripts/bp_debug.py [case]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from maskclustering_amd import _native  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "s1_tiny"
z = dict(np.load(os.path.join(REPO, "tests", "golden", name + ".npz")))
ctx = _native.Context(0)
print("device CUs", ctx.num_cu if hasattr(ctx, "num_cu") else "?", file=sys.stderr, flush=True)
ctx.set_points(np.asarray(z["in_scene"], np.float64).astype(np.float32))
ctx.backproject(z["in_depth"], z["in_seg"], z["in_intrinsics"], z["in_poses"])
col, lab, off, pts = ctx.bp_masks()
print("masks", len(col), "points", len(pts), flush=True)
