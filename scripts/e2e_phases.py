"""Diagnostic: host wall time of each call of one single-GPU C3 E2E step (the bench default at
N = 1), to locate host time between the device groups.

    python scripts/e2e_phases.py [shape] [steps]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import maskclustering_amd  # noqa: E402,F401
import numpy as np  # noqa: E402
import torch  # noqa: E402

from maskclustering_amd import _native  # noqa: E402
from maskclustering_amd.pipeline import GraphRun  # noqa: E402
from maskclustering_amd.synthetic_frames import make_frames_shape  # noqa: E402

shape = sys.argv[1] if len(sys.argv) > 1 else "c3"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
CFG = dict(mask_visible_threshold=0.3, undersegment_filter_threshold=0.3, view_consensus_threshold=0.9,
           contained_threshold=0.8)
fr = make_frames_shape(shape, seed=0, device="cuda:0", out="torch")
dev = torch.device("cuda", 0)
run = GraphRun(0)
ctx = run.ctx
ctx.set_stream(torch.cuda.current_stream().cuda_stream)
scene = torch.tensor(fr.scene_points, dtype=torch.float32, device=dev)
ctx.set_points(device_ptr=scene.data_ptr(), num_points=fr.num_points)
K = torch.from_numpy(np.ascontiguousarray(fr.intrinsics)).to(dev)
T = torch.from_numpy(np.ascontiguousarray(fr.poses.reshape(-1, 16))).to(dev)
prm = _native.bp_params()
F, H, W = fr.depth.shape
for it in range(steps):
    torch.cuda.synchronize()
    t = [time.perf_counter()]
    ctx.backproject(None, None, None, None, prm, shape=(F, H, W),
                    device_ptrs=(fr.depth.data_ptr(), fr.seg.data_ptr(), K.data_ptr(), T.data_ptr()))
    t.append(time.perf_counter())
    col, lab, off = ctx.bp_mask_index()
    t.append(time.perf_counter())
    ctx.use_backprojection()
    t.append(time.perf_counter())
    run.build(CFG["mask_visible_threshold"], CFG["contained_threshold"], CFG["undersegment_filter_threshold"])
    torch.cuda.synchronize()
    t.append(time.perf_counter())
    run.cluster(CFG["view_consensus_threshold"])
    torch.cuda.synchronize()
    t.append(time.perf_counter())
    names = ["backproject", "mask_index", "use_backprojection", "build (S2-S5)", "cluster (S6-S7)"]
    print(f"step {it}: total {1e3 * (t[-1] - t[0]):.1f} ms  " +
          "  ".join(f"{n} {1e3 * (b - a):.2f}" for n, a, b in zip(names, t, t[1:])), flush=True)
