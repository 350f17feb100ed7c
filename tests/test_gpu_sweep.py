"""The scene-parallel sweep (BASELINE configs[4]; the reference's run.py:33-50: one process per GPU,
scene i on rank i mod N, main.py's path per scene) through maskclustering_amd.sweep, as bench.py
--variant sweep runs it: distinct scenes one after another on one context (each scene's points set,
so its ball-query grid is rebuilt; the S1 batches sized from the scenes before), every scene's S1
masks and S2-S6 outputs equal to the oracle's for that scene alone."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

KEYS = ["gl_col", "gl_label", "boundary", "vf_bits", "c_row", "c_col", "undersegment", "node0_g", "thr_value",
        "thr_is_int", "num_iters", "level_sizes", "edge_counts", "obj_mask_off", "obj_mask_idx", "obj_pt_off",
        "obj_pt_idx", "obj_vf_bits", "obj_c_off", "obj_c_idx", "obj_node_info"]


def test_sweep_scenes_each_equal_the_oracle():
    import torch
    from maskclustering_amd.dataset_configs import graph_thresholds
    from maskclustering_amd.sweep import SceneSweep
    from maskclustering_amd.synthetic_frames import make_frames_shape
    cfg = graph_thresholds("scannet")
    dev = torch.device("cuda", 0)
    sw = SceneSweep(0, cfg, stream=torch.cuda.current_stream().cuda_stream)
    # distinct scenes (different points, frames, sizes), a repeat of the first at the end
    scenes = [("small", 0), ("small", 1), ("tiny", 2), ("small", 3), ("small", 0)]
    for shape, seed in scenes:
        fr = make_frames_shape(shape, seed=seed)
        t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a)).to(dev, dt)  # noqa: E731
        pts = t(fr.scene_points, torch.float32)
        objects = sw.run_scene(pts, t(fr.depth, torch.float32), t(fr.seg, torch.uint8), t(fr.intrinsics, torch.float64),
                               t(fr.poses.reshape(-1, 16), torch.float64))
        s1 = oracle.s1_frames(fr.scene_points.astype(np.float32), fr.depth, fr.seg, fr.intrinsics, fr.poses)
        col = np.concatenate([np.full(len(r[0]), c, np.int32) for c, r in enumerate(s1)])
        lab = np.concatenate([r[0] for r in s1]).astype(np.int32)
        off = np.concatenate([[0], np.cumsum(np.concatenate([np.diff(r[1]) for r in s1]))]).astype(np.int64)
        opts = np.concatenate([r[2] for r in s1]).astype(np.int32)
        dcol, dlab, doff, dpts = sw.ctx.bp_masks()
        for a, b, k in ((dcol, col, "col"), (dlab, lab, "label"), (doff, off, "off"), (dpts, opts, "pts")):
            np.testing.assert_array_equal(a, b, err_msg=f"{shape}/{seed} S1 {k}")
        want = oracle.run_sparse(fr.num_points, fr.num_frames, col, lab, off, opts, **cfg)
        got = sw.run.canonical(dense=False)
        for k in KEYS:
            np.testing.assert_array_equal(np.asarray(got[k]), np.asarray(want[k]), err_msg=f"{shape}/{seed} {k}")
        assert objects == len(want["obj_mask_off"]) - 1
