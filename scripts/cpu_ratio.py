"""CPU context ratio of SURVEY.md §8(d)(ii): the reference's own S2-S6 (imported unmodified
through the Appendix B harness of tests/golden/make_golden.py) against the build's C port
(oracle/mcgraph_oracle.c) on the SAME synthetic C2 scene, both on this container's cores.

Run ONLY in the build container (it imports /root/reference):

    python scripts/cpu_ratio.py [shape] [seed]

Writes profiles/cpu_ratio_<shape>.json, which bench.py quotes in cpu_baseline (the reference
itself never travels to the GPU box).
"""
from __future__ import annotations

import json
import os
import sys
import time
from types import SimpleNamespace

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))

CFG = dict(mask_visible_threshold=0.3, undersegment_filter_threshold=0.3, view_consensus_threshold=0.9,
           contained_threshold=0.8)  # configs/scannet.json


def time_reference(scene):
    import make_golden as mg
    construction, iterative_clustering, nx, torch = mg._import_reference()
    per_frame = scene.per_frame_dicts(list(range(scene.num_frames)))
    construction.frame_backprojection = lambda ds, sp, fid: (
        per_frame[fid], list(set().union(*per_frame[fid].values())) if per_frame[fid] else [])
    args = SimpleNamespace(debug=False, **CFG)
    sp = np.zeros((scene.num_points, 3))
    fl = list(range(scene.num_frames))
    tm = {}
    t = time.perf_counter()
    boundary, pim, mpc, pfm, gl = construction.build_point_in_mask_matrix(args, sp, fl, None)
    tm["s2"] = time.perf_counter() - t
    t = time.perf_counter()
    vf, cm, us = construction.process_masks(fl, gl, pim, boundary, mpc, args)
    tm["s3"] = time.perf_counter() - t
    t = time.perf_counter()
    thr = construction.get_observer_num_thresholds(vf)
    nodes = construction.init_nodes(gl, vf, cm, us, mpc)
    tm["s4_s5"] = time.perf_counter() - t
    t = time.perf_counter()
    objs = iterative_clustering.iterative_clustering(nodes, thr, args.view_consensus_threshold, False)
    tm["s6"] = time.perf_counter() - t
    tm["objects"] = len(objs)
    tm["threads"] = torch.get_num_threads()
    return tm


def main():
    from maskclustering_amd.synthetic import make_shape
    from oracle import oracle
    shape = sys.argv[1] if len(sys.argv) > 1 else "c2"
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    scene = make_shape(shape, seed=seed)
    best = None
    for _ in range(3):
        tm = {}
        oracle.run(scene.num_points, scene.num_frames, scene.mask_col, scene.mask_label, scene.mask_off,
                   scene.mask_pts, timings=tm, **CFG)
        tot = tm["s2"] + tm["s3"] + tm["s4"] + tm["s6"]
        if best is None or tot < best[0]:
            best = (tot, tm)
    ref = time_reference(scene)
    ref_tot = ref["s2"] + ref["s3"] + ref["s4_s5"] + ref["s6"]
    out = {"shape": shape, "seed": seed, "M": scene.num_masks, "host_cores": os.cpu_count(),
           "reference_s": round(ref_tot, 2), "reference_stages_s": {k: round(v, 3) for k, v in ref.items()
                                                                   if k.startswith("s")},
           "reference_torch_threads": ref["threads"],
           "port_s": round(best[0], 3), "port_threads": best[1]["threads"],
           "port_stages_s": {k: round(best[1][k], 3) for k in ("s2", "s3", "s4", "s6")},
           "reference_over_port": round(ref_tot / best[0], 1)}
    path = os.path.join(REPO, "profiles", f"cpu_ratio_{shape}.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
