mkdir -p gpurun_out/abl
for L in libmcgraph.so libmcgraph_abl1.so libmcgraph_abl2.so libmcgraph_abl3.so libmcgraph_abl4.so; do
  MCGRAPH_LIB=maskclustering_amd/$L timeout -k 10 200 python - >> gpurun_out/abl/out.txt 2>&1 <<'PY'
import os, sys, time
sys.path.insert(0, '.')
import numpy as np, torch
from maskclustering_amd import _native
from maskclustering_amd.synthetic_frames import make_frames_shape
fr = make_frames_shape("c2", seed=0, device="cuda")
ctx = _native.Context(0)
ctx.set_points(fr.scene_points.astype(np.float32))
for rep in range(3):
    ctx.set_timing(True); ctx.reset_kernel_times()
    ctx.backproject(fr.depth, fr.seg, fr.intrinsics, fr.poses)
    ctx.synchronize()
print(os.environ["MCGRAPH_LIB"], {g: round(ctx.kernel_time(g)[0], 3) for g in ("bp_pixels", "bp_voxel", "bp_denoise", "bp_query")})
PY
done
cat gpurun_out/abl/out.txt | grep -v amdgpu.ids
