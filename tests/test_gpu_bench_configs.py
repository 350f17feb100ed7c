"""Parity on the scenes bench.py measures (BASELINE configs[1] and configs[2]), the HIP path through
the C-ABI against the CPU oracle, bit for bit:

* ``c2_e2e``: the whole C2 RGB-D scene (250 frames 640x480, P ~ 240k, M ~ 15k) S1 -> S6 on the device
  against oracle/s1_oracle.c (OpenMP over frames) feeding the dense S2-S6 oracle
  (oracle/mcgraph_oracle.c); every canonical stage, the per-candidate S1 statistics and the mask CSR.
* ``c3_s1``: three 16-frame windows (first, middle, last) of the C3 scene at 1920x1440 through
  mc_backproject against the oracle's S1, per candidate mask statistics and neighbour sets.
* ``c3_e2e``: the full C3 scene as the bench runs it (1500 frames resident in HBM, S1 -> S6): every
  frame's S1 against the oracle's, then S2-S6 against the sparse oracle (oracle/graph_sparse.c) on
  that mask set, under configs/scannetpp.json's thresholds (the bench's C3 line) and scannet's.
* ``c4``: the Matterport-region-shaped scene (BASELINE configs[3]: 2000 frames of 1280x1024, depth in
  1/4000 m units, ~120k masks): the whole scene S1 -> S6 on the device, every frame's S1 against the
  oracle's (100 frames at a time), then S2-S6 against the sparse oracle on the device's mask set.

The oracle is pinned to the reference's own outputs by tests/test_s1_oracle.py and
tests/test_oracle_golden.py; the Open3D / pytorch3d arithmetic inside S1 is parity unpinned
(DESIGN.md §2.2)."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

from maskclustering_amd.dataset_configs import graph_thresholds

CFG = graph_thresholds("scannet")  # C2 = the ScanNet-shaped scene
# oracle stats columns: id npix nvox ndbscan nsor ncand ncovered nneighbors kept
# device stats columns: frame id npix nvox ndbscan nsor -1 ncovered nneighbors kept
CMP_COLS = [(1, 0), (2, 1), (3, 2), (4, 3), (5, 4), (7, 6), (8, 7), (9, 8)]


def _compare_s1(dev_masks, dev_stats, want, frame_ids):
    """device CSR (col, label, off, pts) + candidate stats against the oracle's per-frame results"""
    col, lab, off, pts = dev_masks
    g = 0
    for c, (f, (ol, oo, op, ost)) in enumerate(zip(frame_ids, want)):
        big = ost[ost[:, 1] >= 25]
        dev = dev_stats[dev_stats[:, 0] == c]
        assert len(dev) == len(big), f"frame {f}: candidates {len(dev)} vs {len(big)}"
        for dc, oc in CMP_COLS:
            np.testing.assert_array_equal(dev[:, dc], big[:, oc], err_msg=f"frame {f} stat column {dc}")
        for k in range(len(ol)):
            assert col[g] == c and lab[g] == ol[k], (f, k)
            np.testing.assert_array_equal(pts[off[g]:off[g + 1]], op[oo[k]:oo[k + 1]], err_msg=f"frame {f} id {ol[k]}")
            g += 1
    assert g == len(col)


def test_c2_e2e_matches_oracle():
    from golden_compare import assert_matches
    from maskclustering_amd.pipeline import GraphRun
    from maskclustering_amd.synthetic_frames import make_frames_shape
    fr = make_frames_shape("c2", seed=0, device="cuda:0")
    assert fr.depth.shape == (250, 480, 640)
    scene = fr.scene_points.astype(np.float32)
    run = GraphRun(0)
    ctx = run.ctx
    ctx.set_points(scene)
    ctx.backproject(fr.depth, fr.seg, fr.intrinsics, fr.poses)
    masks = ctx.bp_masks()
    stats = ctx.bp_candidates()
    s1 = oracle.s1_frames(scene, fr.depth, fr.seg, fr.intrinsics, fr.poses)
    _compare_s1(masks, stats, s1, range(fr.num_frames))
    col, lab, off, pts = masks
    assert len(col) > 12_000
    run.P, run.F = fr.num_points, fr.num_frames
    run.mask_col, run.mask_label = col, lab
    ctx.use_backprojection()
    run.step(**CFG)
    want = oracle.run(fr.num_points, fr.num_frames, col.astype(np.int32), lab.astype(np.int32),
                      np.asarray(off, np.int64), np.asarray(pts, np.int32), **CFG)
    assert_matches(run.canonical(), want)


def _compare_every_frame(fr, masks, stats, chunk=100):
    """S1 of every frame of a device-resident scene (torch frames) against the oracle's, `chunk`
    frames at a time through the host"""
    F = fr.depth.shape[0]
    scene = fr.scene_points.astype(np.float32)
    col_all = masks[0]
    for f0 in range(0, F, chunk):
        f1 = min(F, f0 + chunk)
        want = oracle.s1_frames(scene, fr.depth[f0:f1].cpu().numpy(), fr.seg[f0:f1].cpu().numpy(),
                                fr.intrinsics[f0:f1], fr.poses[f0:f1])
        g0, g1 = np.searchsorted(col_all, [f0, f1])
        o0 = masks[2][g0]
        sub = (col_all[g0:g1] - f0, masks[1][g0:g1], masks[2][g0:g1 + 1] - o0, masks[3][o0:masks[2][g1]])
        st = stats[(stats[:, 0] >= f0) & (stats[:, 0] < f1)].copy()
        st[:, 0] -= f0
        _compare_s1(sub, st, want, range(f0, f1))


def test_c3_s1_windows_match_oracle():
    from maskclustering_amd import _native
    from maskclustering_amd.synthetic_frames import FRAME_SHAPES, make_frames_shape
    F = FRAME_SHAPES["c3"]["num_frames"]
    frames = [*range(0, 16), *range(F // 2 - 8, F // 2 + 8), *range(F - 16, F)]
    fr = make_frames_shape("c3", seed=0, device="cuda:0", frames=frames)
    assert fr.depth.shape == (48, 1440, 1920)
    scene = fr.scene_points.astype(np.float32)
    ctx = _native.Context(0)
    ctx.set_points(scene)
    ctx.backproject(fr.depth, fr.seg, fr.intrinsics, fr.poses)
    s1 = oracle.s1_frames(scene, fr.depth, fr.seg, fr.intrinsics, fr.poses)
    _compare_s1(ctx.bp_masks(), ctx.bp_candidates(), s1, frames)


def test_c3_e2e_matches_oracle():
    """the bench's own C3 step (frames resident in HBM, S1 -> S6), every stage against the oracle"""
    import torch
    from maskclustering_amd import _native
    from maskclustering_amd.pipeline import GraphRun
    from maskclustering_amd.synthetic_frames import make_frames_shape
    fr = make_frames_shape("c3", seed=0, device="cuda:0", out="torch")
    dev = torch.device("cuda", 0)
    t_scene = torch.tensor(fr.scene_points, dtype=torch.float32, device=dev)
    t_K = torch.from_numpy(np.ascontiguousarray(fr.intrinsics)).to(dev)
    t_T = torch.from_numpy(np.ascontiguousarray(fr.poses.reshape(-1, 16))).to(dev)
    run = GraphRun(0)
    ctx = run.ctx
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    ctx.set_points(device_ptr=t_scene.data_ptr(), num_points=fr.num_points)
    F, H, W = fr.depth.shape
    ctx.backproject(None, None, None, None, _native.bp_params(), shape=(F, H, W),
                    device_ptrs=(fr.depth.data_ptr(), fr.seg.data_ptr(), t_K.data_ptr(), t_T.data_ptr()))
    masks = ctx.bp_masks()
    _compare_every_frame(fr, masks, ctx.bp_candidates())
    col, lab, off, pts = masks
    del fr
    torch.cuda.empty_cache()
    assert len(col) > 70_000
    run.P, run.F = len(t_scene), F
    run.mask_col, run.mask_label = col, lab
    # S2-S6 under the ScanNet++ config the bench's C3 line runs (configs/scannetpp.json: ct = 1, whose
    # edge rule needs S >= 2 at O = 1), then under configs/scannet.json, on the same resident masks
    for ds in ("scannetpp", "scannet"):
        cfg = graph_thresholds(ds)
        ctx.use_backprojection()
        run.step(**cfg)
        _assert_graph_matches(run, len(t_scene), F, col, lab, off, pts, cfg, ds)


def _assert_graph_matches(run, P, F, col, lab, off, pts, cfg, what):
    got = run.canonical(dense=False)
    want = oracle.run_sparse(P, F, col.astype(np.int32), lab.astype(np.int32), np.asarray(off, np.int64),
                             np.asarray(pts, np.int32), **cfg)
    for k in ["gl_col", "gl_label", "boundary", "vf_bits", "c_row", "c_col", "undersegment", "node0_g", "thr_value",
              "thr_is_int", "num_iters", "level_sizes", "edge_counts", "obj_mask_off", "obj_mask_idx", "obj_pt_off",
              "obj_pt_idx", "obj_vf_bits", "obj_c_off", "obj_c_idx", "obj_node_info"]:
        np.testing.assert_array_equal(np.asarray(got[k]), np.asarray(want[k]), err_msg=f"{what}: {k}")
    for t in range(int(want["num_iters"])):
        np.testing.assert_array_equal(got[f"part_{t}"], want[f"part_{t}"], err_msg=f"{what}: partition {t}")


def _c4_frames_window():
    from maskclustering_amd.synthetic_frames import FRAME_SHAPES
    F = FRAME_SHAPES["c4"]["num_frames"]
    return [*range(0, 16), *range(F // 2 - 8, F // 2 + 8), *range(F - 16, F)]


def test_c4_s1_windows_match_oracle():
    from maskclustering_amd import _native
    from maskclustering_amd.synthetic_frames import make_frames_shape
    frames = _c4_frames_window()
    fr = make_frames_shape("c4", seed=0, device="cuda:0", frames=frames)
    assert fr.depth.shape == (48, 1024, 1280)
    scene = fr.scene_points.astype(np.float32)
    ctx = _native.Context(0)
    ctx.set_points(scene)
    ctx.backproject(fr.depth, fr.seg, fr.intrinsics, fr.poses)
    s1 = oracle.s1_frames(scene, fr.depth, fr.seg, fr.intrinsics, fr.poses)
    _compare_s1(ctx.bp_masks(), ctx.bp_candidates(), s1, frames)


def test_c4_e2e_matches_oracle():
    """the whole C4 scene S1 -> S6 on the device (frames resident in HBM): every frame's S1 against the
    oracle, then S2-S6 against the sparse oracle on the device's mask set"""
    import torch
    from maskclustering_amd import _native
    from maskclustering_amd.pipeline import GraphRun
    from maskclustering_amd.synthetic_frames import make_frames_shape
    fr = make_frames_shape("c4", seed=0, device="cuda:0", out="torch")
    dev = torch.device("cuda", 0)
    t_scene = torch.tensor(fr.scene_points, dtype=torch.float32, device=dev)
    t_K = torch.from_numpy(np.ascontiguousarray(fr.intrinsics)).to(dev)
    t_T = torch.from_numpy(np.ascontiguousarray(fr.poses.reshape(-1, 16))).to(dev)
    run = GraphRun(0)
    ctx = run.ctx
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    ctx.set_points(device_ptr=t_scene.data_ptr(), num_points=fr.num_points)
    F, H, W = fr.depth.shape
    ctx.backproject(None, None, None, None, _native.bp_params(), shape=(F, H, W),
                    device_ptrs=(fr.depth.data_ptr(), fr.seg.data_ptr(), t_K.data_ptr(), t_T.data_ptr()))
    masks = ctx.bp_masks()
    # S1 of every one of the 2000 frames (1280x1024, depth in 1/4000 m) against the oracle's
    _compare_every_frame(fr, masks, ctx.bp_candidates())
    col, lab, off, pts = masks
    del fr
    torch.cuda.empty_cache()
    assert len(col) > 100_000
    run.P, run.F = len(t_scene), F
    run.mask_col, run.mask_label = col, lab
    cfg = graph_thresholds("matterport3d")  # configs/matterport3d.json
    ctx.use_backprojection()
    run.step(**cfg)
    _assert_graph_matches(run, len(t_scene), F, col, lab, off, pts, cfg, "matterport3d")
