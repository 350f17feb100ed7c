"""Runs of equal voxel keys in the slots' pixel lists (row-major mask pixels with valid depth, cut at
every 64th pixel as the voxel kernel's waves cut them), voxels per slot and the share of slots and
pixels by voxel count, on a few frames of a synthetic scene (numpy, CPU; DESIGN.md §4 bp_voxel).

    python scripts/voxel_runs.py [shape] [first frame] [frames] [step]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from maskclustering_amd.synthetic_frames import make_frames_shape  # noqa: E402


def main():
    shape = sys.argv[1] if len(sys.argv) > 1 else "c3"
    f0 = int(sys.argv[2]) if len(sys.argv) > 2 else 600
    nf = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    step = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    fr = make_frames_shape(shape, seed=0, frames=list(range(f0, f0 + nf * step, step)))
    H, W = fr.depth.shape[1:]
    rows = []
    for f in range(fr.depth.shape[0]):
        d = fr.depth[f].astype(np.float64)
        s = fr.seg[f]
        K, T = fr.intrinsics[f], fr.poses[f]
        v, u = np.mgrid[0:H, 0:W]
        P = np.stack([((u - K[2]) * d) / K[0], ((v - K[3]) * d) / K[1], d, np.ones_like(d)], -1) @ T.T
        for m in np.unique(s):
            if m == 0:
                continue
            idx = np.nonzero(((s == m) & (d > 0)).reshape(-1))[0]
            if len(idx) < 25:
                continue
            p = P.reshape(-1, 4)[idx, :3]
            key = np.floor((p - (p.min(0) - 0.005)) / 0.01).astype(np.int64)
            kk = key[:, 0] * (1 << 42) + key[:, 1] * (1 << 21) + key[:, 2]
            head = (np.arange(len(idx)) % 64 == 0) | np.r_[True, kk[1:] != kk[:-1]]
            rows.append((len(idx), int(head.sum()), len(np.unique(kk))))
    a = np.array(rows, np.float64)
    print(f"{shape} frames {f0}..{f0 + (nf - 1) * step} step {step}: slots {len(a)}, pixels/slot {a[:, 0].mean():.0f}, "
          f"runs/slot {a[:, 1].mean():.0f}, pixels/run {a[:, 0].sum() / a[:, 1].sum():.2f}, voxels/slot {a[:, 2].mean():.0f}, "
          f"runs/voxel {a[:, 1].sum() / a[:, 2].sum():.2f}")
    for lim in (512, 1024, 2048, 4096):
        sel = a[:, 2] <= lim
        print(f"  voxels <= {lim}: {sel.mean():.3f} of the slots, {a[sel, 0].sum() / a[:, 0].sum():.3f} of the pixels")


if __name__ == "__main__":
    main()
