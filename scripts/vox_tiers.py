"""Diagnostic: the slots of a bench scene that overflow the first voxel tier (more than 2048 voxels),
their pixel and voxel counts, and the pixel-count thresholds that would predict them.

    python scripts/vox_tiers.py [shape] [first frame] [frames]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from maskclustering_amd import _native  # noqa: E402
from maskclustering_amd.synthetic_frames import make_frames_shape  # noqa: E402

shape = sys.argv[1] if len(sys.argv) > 1 else "c3"
f0 = int(sys.argv[2]) if len(sys.argv) > 2 else 0
nf = int(sys.argv[3]) if len(sys.argv) > 3 else 750
fr = make_frames_shape(shape, seed=0, device="cuda", frames=range(f0, f0 + nf))
ctx = _native.Context(0)
ctx.set_points(fr.scene_points.astype(np.float32))
ctx.backproject(fr.depth, fr.seg, fr.intrinsics, fr.poses)
ctx.synchronize()
st = ctx.bp_candidates()
npix, nvox = st[:, 2].astype(np.int64), st[:, 3].astype(np.int64)
print("slots", len(st), "pixels", int(npix.sum()), "voxels", int(nvox.sum()))
big = nvox > 2048
print("tier-2 slots (nvox > 2048):", int(big.sum()), "pixels", int(npix[big].sum()),
      f"({npix[big].sum() / npix.sum():.3f} of all), voxels", int(nvox[big].sum()))
if big.any():
    print("  their npix: min", int(npix[big].min()), "p50", int(np.median(npix[big])), "max", int(npix[big].max()))
    print("  their nvox: min", int(nvox[big].min()), "p50", int(np.median(nvox[big])), "max", int(nvox[big].max()))
for thr in (8192, 16384, 32768, 65536, 131072):
    sel = npix >= thr
    print(f"npix >= {thr:6d}: {int(sel.sum()):5d} slots, of them tier-2 {int((sel & big).sum()):5d};"
          f" tier-2 slots below: {int((big & ~sel).sum())}")
top = np.argsort(-npix)[:10]
print("largest slots by pixels (npix, nvox):", [(int(npix[i]), int(nvox[i])) for i in top])
