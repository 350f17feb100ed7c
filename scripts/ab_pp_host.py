"""A/B of post_process_objects' host query building on one C2 scene, in one process: the bulk pass
(_bulk_columns) against the per-node walk (bulk forced off), alternating, plus the S6 fast-path check.
Prints one JSON line.  GPU run: python scripts/ab_pp_host.py"""
import json
import os
import sys
import time
from types import SimpleNamespace

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from maskclustering_amd.graph import construction, iterative_clustering  # noqa: E402
from maskclustering_amd.synthetic_frames import make_frames_shape  # noqa: E402
from maskclustering_amd.utils import post_process as pp  # noqa: E402


def main():
    import torch
    fr = make_frames_shape("c2", seed=0, device="cuda:0")
    fids = [int(x) for x in np.arange(0, 10 * fr.num_frames, 10)]
    args = SimpleNamespace(debug=False, point_filter_threshold=0.5, **bench.CFG)
    ds = bench.FrameDataset(fr, fids, raw_depth=True)
    nodes, thr, mpc, pfm = construction.mask_graph_construction(args, fr.scene_points, fids, ds)
    t = time.perf_counter()
    for _ in range(50):
        assert iterative_clustering._fast_path(nodes) is not None
    fast_ms = (time.perf_counter() - t) / 50 * 1e3
    objects = iterative_clustering.iterative_clustering(nodes, thr, args.view_consensus_threshold, False)
    bulk = pp._bulk_columns
    res = {"bulk": [], "per_node": []}
    ref = None
    for i in range(24):
        mode = "bulk" if i % 2 else "per_node"
        pp._bulk_columns = bulk if mode == "bulk" else (lambda *a: None)
        torch.cuda.synchronize()
        t = time.perf_counter()
        out = pp.post_process_objects(objects, mpc, fr.scene_points, pfm, fids, args.point_filter_threshold)
        torch.cuda.synchronize()
        res[mode].append((time.perf_counter() - t) * 1e3)
        key = ([o.tolist() for o in out[0]], out[1])
        if ref is None:
            ref = key
        assert key == ref, "bulk and per-node query building disagree"
    pp._bulk_columns = bulk
    import cProfile
    import pstats
    pr = cProfile.Profile()
    pr.enable()
    pp.post_process_objects(objects, mpc, fr.scene_points, pfm, fids, args.point_filter_threshold)
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr, stream=sys.stderr).sort_stats("tottime").print_stats(25)
    print(json.dumps({"what": "post_process_objects wall ms on C2 (870 objects), bulk vs per-node host query building; "
                              "S6 fast-path check ms on 14k level-0 nodes",
                      "bulk_ms_median": float(np.median(res["bulk"][2:])),
                      "per_node_ms_median": float(np.median(res["per_node"][2:])),
                      "bulk_ms": [round(x, 2) for x in res["bulk"]],
                      "per_node_ms": [round(x, 2) for x in res["per_node"]],
                      "fast_path_check_ms": round(fast_ms, 3), "outputs_identical": True}), flush=True)


if __name__ == "__main__":
    main()
