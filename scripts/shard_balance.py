"""Frame-slice balance on one GPU: the S1 time of each rank's slice of a bench scene, for equal
frame counts (frame_slice) and for cost-balanced slices (balanced_frame_slices over frame_costs),
at world sizes 2, 4 and 8.  Each slice is back-projected alone, as its rank would, and timed with
a device synchronisation on both sides (best of 3).  The ratio max / mean over the ranks is the strong-scaling
loss the slicing leaves.

    python scripts/shard_balance.py [shape]
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from maskclustering_amd import _native  # noqa: E402
from maskclustering_amd.frame_shard import balanced_frame_slices, frame_costs, frame_slice  # noqa: E402
from maskclustering_amd.synthetic_frames import make_frames_shape  # noqa: E402


def main():
    shape = sys.argv[1] if len(sys.argv) > 1 else "c3"
    t0 = time.perf_counter()
    fr = make_frames_shape(shape, seed=0, device="cuda:0", out="torch")
    print(f"rendered {fr.num_frames} frames in {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
    dev = torch.device("cuda", 0)
    ctx = _native.Context(0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    scene = torch.tensor(fr.scene_points, dtype=torch.float32, device=dev)
    ctx.set_points(device_ptr=scene.data_ptr(), num_points=fr.num_points)
    K = torch.from_numpy(np.ascontiguousarray(fr.intrinsics)).to(dev)
    T = torch.from_numpy(np.ascontiguousarray(fr.poses.reshape(-1, 16))).to(dev)
    F, H, W = fr.depth.shape
    prm = _native.bp_params()
    costs = frame_costs(fr.depth, fr.seg, fr.intrinsics).cpu().numpy()

    def s1_ms(lo, hi):
        if hi <= lo:
            return 0.0
        args = dict(shape=(hi - lo, H, W), device_ptrs=(fr.depth[lo].data_ptr(), fr.seg[lo].data_ptr(),
                                                         K[lo].data_ptr(), T[lo].data_ptr()))
        ctx.backproject(None, None, None, None, prm, **args)
        torch.cuda.synchronize()
        best = 1e30
        for _ in range(3):
            t = time.perf_counter()
            ctx.backproject(None, None, None, None, prm, **args)
            torch.cuda.synchronize()
            best = min(best, 1e3 * (time.perf_counter() - t))
        return best

    out = {"shape": shape, "frames": F, "cost_total": float(costs.sum()), "worlds": {}}
    for world in (2, 4, 8):
        rec = {}
        for name, sl in (("equal", [frame_slice(F, world, r) for r in range(world)]),
                         ("balanced", balanced_frame_slices(costs, world))):
            ms = [s1_ms(lo, hi) for lo, hi in sl]
            rec[name] = {"slices": sl, "s1_ms": [round(x, 3) for x in ms],
                         "cost_share": [round(float(costs[lo:hi].sum() / costs.sum()), 4) for lo, hi in sl],
                         "max_over_mean": round(max(ms) / (sum(ms) / len(ms)), 4)}
            print(f"world {world} {name}: max/mean {rec[name]['max_over_mean']} ms {rec[name]['s1_ms']}",
                  file=sys.stderr, flush=True)
        out["worlds"][world] = rec
    out["s1_ms_whole"] = round(s1_ms(0, F), 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
