"""Per-group kernel timing of one library build (MCGRAPH_LIB selects a profiling
variant).  Prints build groups (S2-S4) and first-iteration S6 groups, in us."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from maskclustering_amd.pipeline import GraphRun  # noqa: E402
from maskclustering_amd.synthetic import make_shape  # noqa: E402

shape = sys.argv[1] if len(sys.argv) > 1 else "c2"
reps = 10
scene = make_shape(shape, seed=0)
run = GraphRun(0)
run.set_scene(scene)
cfg = (0.3, 0.8, 0.3)
for _ in range(3):
    run.build(*cfg)
thr, _ = run.ctx.thresholds()
groups_b = ["s2_point_lists", "s3_masks", "s3_undo_s5", "s4_observer_hist"]
groups_c = ["s6_columns", "s6_pairs", "s6_components", "s6_merge", "s7_points"]
run.ctx.reset_kernel_times()
run.ctx.set_timing(True)
for _ in range(reps):
    run.build(*cfg)
run.ctx.synchronize()
out = {g: round(run.ctx.kernel_time(g)[0] / reps * 1e3, 1) for g in groups_b}
for _ in range(3):
    run.cluster(0.9, thresholds=thr[:1])
run.ctx.synchronize()
run.ctx.reset_kernel_times()
for _ in range(reps):
    run.cluster(0.9, thresholds=thr[:1])
run.ctx.synchronize()
out.update({g + "@it0": round(run.ctx.kernel_time(g)[0] / reps * 1e3, 1) for g in groups_c})
print(json.dumps({"lib": os.path.basename(os.environ.get("MCGRAPH_LIB", "libmcgraph.so")), **out}))
