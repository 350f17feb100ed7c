"""Diagnostic: S1 of one frame slice of a bench scene (what one rank of an N-rank frame-sharded run
back-projects), wall time against the S1 groups' kernel time, per call.

    python scripts/s1_slice_profile.py [shape] [first frame] [frames] [calls]

Under ``rocprofv3 --kernel-trace`` the last call's dispatch timeline shows where the wall time that
no kernel covers goes (host syncs between the batch's stages, the side streams' tails)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from maskclustering_amd import _native  # noqa: E402
from maskclustering_amd.synthetic_frames import make_frames_shape  # noqa: E402

shape = sys.argv[1] if len(sys.argv) > 1 else "c3"
f0 = int(sys.argv[2]) if len(sys.argv) > 2 else 574
nf = int(sys.argv[3]) if len(sys.argv) > 3 else 181
calls = int(sys.argv[4]) if len(sys.argv) > 4 else 6
t0 = time.perf_counter()
fr = make_frames_shape(shape, seed=0, device="cuda", frames=range(f0, f0 + nf))
print(f"{shape} frames {f0}..{f0 + nf} rendered in {time.perf_counter() - t0:.1f} s", flush=True)
dev = torch.device("cuda", 0)
t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a)).to(dev, dt)  # noqa: E731
depth, seg = t(fr.depth, torch.float32), t(fr.seg, torch.uint8)
K, T = t(fr.intrinsics, torch.float64), t(fr.poses.reshape(-1, 16), torch.float64)
pts = t(fr.scene_points, torch.float32)
ctx = _native.Context(0)
ctx.set_stream(torch.cuda.current_stream().cuda_stream)
prm = _native.bp_params()
groups = ("bp_grid", "bp_pixels", "bp_voxel", "bp_denoise", "bp_query")
F, H, W = depth.shape
# MC_ENVS="A=1;A=2" cycles the calls through environment settings (knobs the library reads per call)
envs = [e for e in os.environ.get("MC_ENVS", "").split(";") if e] or [""]
for c in range(calls):
    tag = envs[c % len(envs)]
    if tag:
        for kv in tag.split(","):
            k, v = kv.split("=")
            os.environ[k] = v
    ctx.set_timing(True)
    ctx.reset_kernel_times()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ctx.set_points(device_ptr=pts.data_ptr(), num_points=len(pts))
    ctx.backproject(None, None, None, None, prm, shape=(F, H, W),
                    device_ptrs=(depth.data_ptr(), seg.data_ptr(), K.data_ptr(), T.data_ptr()))
    ctx.synchronize()
    wall = (time.perf_counter() - t0) * 1e3
    g = {k: round(ctx.kernel_time(k)[0], 2) for k in groups}
    print(f"call {c} [{tag}]: wall {wall:.2f} ms, groups {g}, sum {sum(g.values()):.2f}, batching {ctx.bp_batching()}",
          flush=True)
