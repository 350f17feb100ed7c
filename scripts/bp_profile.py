"""S1 back-projection profile on a frame slice of a synthetic RGB-D shape: per-group device times
and the distribution of the per-slot sizes (pixels, voxels, survivors) the denoise classes see.

    python scripts/bp_profile.py [shape] [first_frame] [num_frames] [repeats]
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from maskclustering_amd import _native  # noqa: E402
from maskclustering_amd.synthetic_frames import make_frames_shape  # noqa: E402


def main():
    shape = sys.argv[1] if len(sys.argv) > 1 else "c3"
    f0 = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    nf = int(sys.argv[3]) if len(sys.argv) > 3 else 100
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    t0 = time.perf_counter()
    fr = make_frames_shape(shape, seed=0, device="cuda:0", frames=range(f0, f0 + nf), out="torch")
    print(f"rendered {nf} frames in {time.perf_counter() - t0:.1f} s", file=sys.stderr)
    dev = torch.device("cuda", 0)
    ctx = _native.Context(0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    scene = torch.tensor(fr.scene_points, dtype=torch.float32, device=dev)
    ctx.set_points(device_ptr=scene.data_ptr(), num_points=fr.num_points)
    K = torch.from_numpy(np.ascontiguousarray(fr.intrinsics)).to(dev)
    T = torch.from_numpy(np.ascontiguousarray(fr.poses.reshape(-1, 16))).to(dev)
    F, H, W = fr.depth.shape
    prm = _native.bp_params()
    run = lambda: ctx.backproject(None, None, None, None, prm, shape=(F, H, W),  # noqa: E731
                                  device_ptrs=(fr.depth.data_ptr(), fr.seg.data_ptr(), K.data_ptr(), T.data_ptr()))
    run()
    torch.cuda.synchronize()
    groups = ["bp_pixels", "bp_voxel", "bp_denoise", "bp_query"]
    ctx.reset_kernel_times()
    ctx.set_timing(True)
    walls = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        run()
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t)
    ctx.set_timing(False)
    st = ctx.bp_candidates()
    nvox, npix, nsor = st[:, 3], st[:, 2], st[:, 5]
    edges = [0, 256, 512, 1024, 2048, 3072, 4096, 8192, 16384, 1 << 30]
    hist = {f"{edges[i]}-{edges[i + 1]}": int(((nvox > edges[i]) & (nvox <= edges[i + 1])).sum())
            for i in range(len(edges) - 1)}
    out = {"shape": shape, "frames": [f0, f0 + nf], "HxW": [H, W], "candidates": int(len(st)),
           "kept": int(ctx.bp_info().num_masks), "wall_ms": round(1e3 * min(walls), 2),
           "group_ms": {g: round(ctx.kernel_time(g)[0] / reps, 3) for g in groups},
           "pixels": {"sum": int(npix.sum()), "mean": float(npix.mean()), "max": int(npix.max())},
           "voxels": {"sum": int(nvox.sum()), "mean": float(nvox.mean()), "p50": float(np.median(nvox)),
                      "p90": float(np.percentile(nvox, 90)), "max": int(nvox.max()), "hist": hist,
                      "voxel_weighted_hist": {k: int(nvox[(nvox > edges[i]) & (nvox <= edges[i + 1])].sum())
                                              for i, k in enumerate(hist)}},
           "survivors": {"sum": int(nsor.sum()), "mean": float(nsor.mean())}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
