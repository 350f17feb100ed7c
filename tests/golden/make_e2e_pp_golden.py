"""Golden fixtures for the whole drop-in path as main.py:17-21 calls it: the REFERENCE's own
``mask_graph_construction`` -> ``iterative_clustering`` -> ``post_process`` (graph/construction.py:7,
graph/iterative_clustering.py:36, utils/post_process.py:173) on the synthetic RGB-D frames of the
api_small fixtures (their stored inputs, so every fixture sees the same frames).

Run ONLY in the build container, where /root/reference exists:

    python tests/golden/make_e2e_pp_golden.py

Open3D / pytorch3d are served by the restatements of make_s1_golden.py (parity of that library
arithmetic unpinned); ``export`` (:148-170, file output only) is replaced by a
capture of its two lists.  Everything else is the reference's unmodified code in one process, so
the CPython set orders it produces (graph/node.py:31-36, :45) are the ones main.py would see.
Stored: the exported objects in order (point ids in the order export receives them, mask lists
with coverages) and, for diagnosis, each final node's ``list(point_ids)`` order.  Data only.
"""
from __future__ import annotations

import os
import sys
from types import SimpleNamespace

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)

import make_api_golden as apig  # noqa: E402
import make_pp_golden as ppg  # noqa: E402
import make_s1_golden as s1g  # noqa: E402

THR = {"scannet": 0.5, "scannetpp": 0.7}  # point_filter_threshold of configs/scannet.json, scannetpp.json


def main():
    mb, torch = s1g._import_reference()
    os.environ["TQDM_DISABLE"] = "1"
    from graph import construction, iterative_clustering  # noqa: E402
    for cfg in ("scannet", "scannetpp"):
        z = dict(np.load(os.path.join(HERE, f"api_small_{cfg}.npz")))
        fr = SimpleNamespace(scene_points=z["in_scene"], depth=z["in_depth"], seg=z["in_seg"],
                             intrinsics=z["in_intrinsics"], poses=z["in_poses"])
        fids = z["in_frame_ids"].tolist()
        ds = apig.FrameDataset(fr, fids, s1g._Intrinsic)
        args = SimpleNamespace(debug=False, **apig.CONFIGS[cfg])
        nodes, thr, mpc, pfm = construction.mask_graph_construction(args, fr.scene_points, list(fids), ds)
        objects = iterative_clustering.iterative_clustering(list(nodes), thr, args.view_consensus_threshold, False)
        orders, got = ppg.run_reference_post_process(objects, mpc, fr.scene_points, pfm, fids, THR[cfg])
        out = {"pp_thr": np.array(THR[cfg])}
        oo, oi, qo, qf, qm, qc = [0], [], [0], [], [], []
        for pts, ml in zip(got["pts"], got["masks"]):
            oi.extend(int(x) for x in pts)
            oo.append(len(oi))
            for f, m, cov in ml:
                qf.append(str(f))
                qm.append(int(m))
                qc.append(float(cov))
            qo.append(len(qm))
        out["obj_pt_off"], out["obj_pt_idx"] = np.array(oo, np.int64), np.array(oi, np.int32)
        out["obj_mask_off"] = np.array(qo, np.int64)
        out["obj_mask_frame"], out["obj_mask_id"] = np.array(qf), np.array(qm, np.int32)
        out["obj_mask_cov"] = np.array(qc, np.float64)
        no, ni = [0], []
        for o in orders:
            ni.extend(int(x) for x in o)
            no.append(len(ni))
        out["node_order_off"], out["node_order_idx"] = np.array(no, np.int64), np.array(ni, np.int32)
        out["node_mask_lists"] = np.array([";".join(f"{f}_{m}" for f, m in o.mask_list) for o in objects])
        path = os.path.join(HERE, f"e2e_pp_small_{cfg}.npz")
        np.savez_compressed(path, **out)
        print(f"{cfg}: nodes={len(objects)} exported objects={len(got['pts'])} "
              f"points={len(oi)} -> {path} {os.path.getsize(path) / 1e3:.1f} kB")
    import json
    import networkx
    with open(os.path.join(HERE, "e2e_pp_small.meta.json"), "w") as f:  # the replay's set orders are networkx 3.x's
        json.dump({"generated_with": {"networkx": networkx.__version__, "numpy": np.__version__},
                   "note": "e2e_pp_small_*.npz: the reference main path run by make_e2e_pp_golden.py; the set-order "
                           "replay reproduces networkx>=3 _plain_bfs orders"}, f, indent=1)


if __name__ == "__main__":
    main()
