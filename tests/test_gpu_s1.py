"""S1 HIP back-projection (mc_backproject) against the reference's own glue
(golden fixtures, tests/golden/make_s1_golden.py) and the CPU restatement
(oracle/s1_oracle.c).  Bit-exact: the outputs are integer sets; the float
steps in between follow the same rounding as the oracle."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

# oracle stats columns: id npix nvox ndbscan nsor ncand ncovered nneighbors kept
# device stats columns: frame id npix nvox ndbscan nsor -1 ncovered nneighbors kept
CMP_COLS = [(1, 0), (2, 1), (3, 2), (4, 3), (5, 4), (7, 6), (8, 7), (9, 8)]


@pytest.fixture(scope="module")
def ctx():
    from maskclustering_amd import _native
    return _native.Context(0)


def _run(ctx, scene, depth, seg, K, T, **prm):
    from maskclustering_amd import _native
    ctx.set_points(np.asarray(scene, np.float64).astype(np.float32))
    ctx.backproject(depth, seg, K, T, _native.bp_params(**prm) if prm else None)
    return ctx.bp_masks()


def _check_against_oracle(ctx, fr, frames=None, **prm):
    from oracle import oracle
    idx = list(range(fr.num_frames)) if frames is None else frames
    col, lab, off, pts = _run(ctx, fr.scene_points, fr.depth[idx], fr.seg[idx], fr.intrinsics[idx], fr.poses[idx],
                              **prm)
    oprm = oracle.BpParams.default(**prm) if prm else None
    st = ctx.bp_candidates()
    scene = fr.scene_points.astype(np.float32)
    g = 0
    row = 0
    for c, f in enumerate(idx):
        ol, oo, op, ost = oracle.s1_frame(scene, fr.depth[f], fr.seg[f], fr.intrinsics[f], fr.poses[f], oprm)
        big = ost[ost[:, 1] >= 25]
        dev = st[st[:, 0] == c]
        assert len(dev) == len(big), f"frame {f}: candidates {len(dev)} vs {len(big)}"
        for dc, oc in CMP_COLS:
            np.testing.assert_array_equal(dev[:, dc], big[:, oc], err_msg=f"frame {f} stat column {dc}")
        row += len(dev)
        for k in range(len(ol)):
            assert col[g] == c and lab[g] == ol[k], (f, k)
            np.testing.assert_array_equal(pts[off[g]:off[g + 1]], op[oo[k]:oo[k + 1]], err_msg=f"frame {f} id {ol[k]}")
            g += 1
    assert g == len(col)


@pytest.mark.parametrize("name", ["s1_tiny", "s1_dense"])
def test_backproject_matches_reference_glue(ctx, name):
    z = dict(np.load(os.path.join(GOLDEN, name + ".npz")))
    col, lab, off, pts = _run(ctx, z["in_scene"], z["in_depth"], z["in_seg"], z["in_intrinsics"], z["in_poses"])
    fo = z["out_frame_off"]
    np.testing.assert_array_equal(lab, z["out_labels"])
    np.testing.assert_array_equal(np.diff(fo), np.bincount(col, minlength=len(fo) - 1))
    np.testing.assert_array_equal(off, z["out_off"])
    np.testing.assert_array_equal(pts, z["out_pts"])


def test_backproject_edge_frames(ctx):
    """inf pose, frames without ids / with tiny masks, ids over invalid depth,
    and the DEPTH_TRUNC pixel that makes the reference raise IndexError."""
    from maskclustering_amd._native import McError, MC_ERR_INVALID
    z = dict(np.load(os.path.join(GOLDEN, "s1_edge.npz")))
    bad = int(np.nonzero(z["out_err"])[0][0])
    with pytest.raises(McError) as e:
        _run(ctx, z["in_scene"], z["in_depth"], z["in_seg"], z["in_intrinsics"], z["in_poses"])
    assert e.value.code == MC_ERR_INVALID and f"frame {bad}" in str(e.value)
    assert ctx.bp_info().error_frame == bad
    keep = [f for f in range(len(z["in_depth"])) if not z["out_err"][f]]
    col, lab, off, pts = _run(ctx, z["in_scene"], z["in_depth"][keep], z["in_seg"][keep], z["in_intrinsics"][keep],
                              z["in_poses"][keep])
    fo = z["out_frame_off"]
    g = 0
    for c, f in enumerate(keep):
        for k in range(fo[f], fo[f + 1]):
            assert col[g] == c and lab[g] == z["out_labels"][k]
            np.testing.assert_array_equal(pts[off[g]:off[g + 1]], z["out_pts"][z["out_off"][k]:z["out_off"][k + 1]])
            g += 1
    assert g == len(col)


@pytest.mark.parametrize("seed", [0, 1])
def test_backproject_stages_match_oracle(ctx, seed):
    from maskclustering_amd.synthetic_frames import make_frames_shape
    fr = make_frames_shape("small", seed=seed)
    _check_against_oracle(ctx, fr)


def test_backproject_dense_frames_match_oracle(ctx):
    """640x480-like pixel density: several pixels per voxel, larger masks."""
    from maskclustering_amd.synthetic_frames import make_frames_shape
    fr = make_frames_shape("tiny", seed=5, H=360, W=480, num_frames=3)
    _check_against_oracle(ctx, fr)


def test_backproject_batched_equals_single(ctx, monkeypatch):
    from maskclustering_amd.synthetic_frames import make_frames_shape
    fr = make_frames_shape("small", seed=2)
    a = _run(ctx, fr.scene_points, fr.depth, fr.seg, fr.intrinsics, fr.poses)
    monkeypatch.setenv("MC_BP_BATCH_PIXELS", str(3 * fr.depth.shape[1] * fr.depth.shape[2]))
    b = _run(ctx, fr.scene_points, fr.depth, fr.seg, fr.intrinsics, fr.poses)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize("frac", ["0.0001", "0.02"])
def test_mask_pixel_capacity_grow_and_redo(ctx, monkeypatch, frac):
    """Batches are sized for the expected share of mask pixels among frame pixels; a batch with more
    mask pixels than that capacity runs no slot, grows the pixel-list arrays and is redone.  Forcing
    a tiny expected share (MC_BP_MASK_FRAC) sends the first batch (of one or of several) down that
    path: the masks and statistics equal the default run's and the oracle's."""
    from maskclustering_amd.synthetic_frames import make_frames_shape
    fr = make_frames_shape("small", seed=6)
    want = _run(ctx, fr.scene_points, fr.depth, fr.seg, fr.intrinsics, fr.poses)
    sw = ctx.bp_candidates()
    for batch in (None, str(4 * fr.depth.shape[1] * fr.depth.shape[2])):
        fresh = _native_ctx()
        monkeypatch.setenv("MC_BP_MASK_FRAC", frac)
        if batch:
            monkeypatch.setenv("MC_BP_BATCH_PIXELS", batch)
        got = _run(fresh, fr.scene_points, fr.depth, fr.seg, fr.intrinsics, fr.poses)
        for x, y in zip(want, got):
            np.testing.assert_array_equal(x, y)
        np.testing.assert_array_equal(sw, fresh.bp_candidates())
        monkeypatch.delenv("MC_BP_MASK_FRAC")
        again = _run(fresh, fr.scene_points, fr.depth, fr.seg, fr.intrinsics, fr.poses)  # sized from the seen share
        for x, y in zip(want, again):
            np.testing.assert_array_equal(x, y)
    _check_against_oracle(ctx, fr)


def _native_ctx():
    from maskclustering_amd import _native
    return _native.Context(0)


@pytest.mark.parametrize("nb", ["1", "3", "16"])
def test_backproject_frames_staged_per_batch(ctx, monkeypatch, nb):
    """mc_backproject_frames (per-frame host arrays, batch b + 1 staged on the copy stream while
    batch b computes) == mc_backproject over the contiguous [F, H, W] arrays."""
    from maskclustering_amd.synthetic_frames import make_frames_shape
    fr = make_frames_shape("small", seed=4)
    a = _run(ctx, fr.scene_points, fr.depth, fr.seg, fr.intrinsics, fr.poses)
    sa = ctx.bp_candidates()
    monkeypatch.setenv("MC_BP_UPLOAD_BATCHES", nb)
    ctx.backproject_frames([np.ascontiguousarray(d) for d in fr.depth], [np.ascontiguousarray(s) for s in fr.seg],
                           fr.intrinsics, fr.poses)
    for x, y in zip(a, ctx.bp_masks()):
        np.testing.assert_array_equal(x, y)
    np.testing.assert_array_equal(sa, ctx.bp_candidates())


@pytest.mark.parametrize("nb", ["1", "3"])
def test_backproject_frames_raw_depth(ctx, monkeypatch, nb):
    """mc_backproject_frames_raw (uint16 frames staged at 2 bytes per pixel, decoded on the copy
    stream, dataset/scannet.py:51-53) == mc_backproject over the float32 frames get_depth returns."""
    from maskclustering_amd.synthetic_frames import make_frames_shape
    fr = make_frames_shape("small", seed=4)
    u16 = np.rint(fr.depth * np.float32(1000.0)).astype(np.uint16)
    assert np.array_equal((u16 / 1000.0).astype(np.float32).view(np.uint32), fr.depth.view(np.uint32))
    a = _run(ctx, fr.scene_points, fr.depth, fr.seg, fr.intrinsics, fr.poses)
    sa = ctx.bp_candidates()
    monkeypatch.setenv("MC_BP_UPLOAD_BATCHES", nb)
    ctx.backproject_frames([np.ascontiguousarray(d) for d in u16], [np.ascontiguousarray(s) for s in fr.seg],
                           fr.intrinsics, fr.poses, depth_scale=1000.0)
    for x, y in zip(a, ctx.bp_masks()):
        np.testing.assert_array_equal(x, y)
    np.testing.assert_array_equal(sa, ctx.bp_candidates())


def test_end_to_end_matches_oracle(ctx):
    """S1 on the device feeding S2-S6 on the device == the oracle's S1 feeding its S2-S6."""
    from maskclustering_amd.pipeline import GraphRun
    from maskclustering_amd.synthetic_frames import make_frames_shape
    from oracle import oracle
    from golden_compare import assert_matches
    fr = make_frames_shape("small", seed=3)
    cfg = dict(mask_visible_threshold=0.3, undersegment_filter_threshold=0.3, view_consensus_threshold=0.9,
               contained_threshold=0.8)
    m = oracle.s1_scene(fr)
    want = oracle.run(fr.num_points, fr.num_frames, m["mask_col"], m["mask_label"], m["mask_off"], m["mask_pts"], **cfg)
    run = GraphRun(0, ctx=ctx)
    ctx.set_points(fr.scene_points.astype(np.float32))
    ctx.backproject(fr.depth, fr.seg, fr.intrinsics, fr.poses)
    col, lab, off, pts = ctx.bp_masks()
    run.P, run.F = fr.num_points, fr.num_frames
    run.mask_col, run.mask_label = col, lab
    ctx.use_backprojection()
    run.step(**cfg)
    assert_matches(run.canonical(), want)


def _check_golden(ctx, name):
    """the reference's own glue output (tests/golden/make_s1_golden.py) for fixture `name`"""
    z = dict(np.load(os.path.join(GOLDEN, name + ".npz")))
    col, lab, off, pts = _run(ctx, z["in_scene"], z["in_depth"], z["in_seg"], z["in_intrinsics"], z["in_poses"])
    fo = z["out_frame_off"]
    np.testing.assert_array_equal(lab, z["out_labels"], err_msg=name)
    np.testing.assert_array_equal(np.diff(fo), np.bincount(col, minlength=len(fo) - 1), err_msg=name)
    np.testing.assert_array_equal(off, z["out_off"], err_msg=name)
    np.testing.assert_array_equal(pts, z["out_pts"], err_msg=name)


def _check_dense(ctx):
    """the dense inputs against their references: the s1_dense fixture against the reference's glue,
    the 360x480 frames against the CPU restatement (every statistics column and every mask)"""
    from maskclustering_amd.synthetic_frames import make_frames_shape
    _check_golden(ctx, "s1_dense")
    _check_against_oracle(ctx, make_frames_shape("tiny", seed=5, H=360, W=480, num_frames=3))


@pytest.mark.parametrize("min_cls", [1, 2, 3, 4, 5, 6])
def test_denoise_size_classes_match_oracle(ctx, monkeypatch, min_cls):
    """Every denoise size class (LDS 512/1024/2048 points, the lean 3072- and 4096-point classes,
    the 16384-point class with every array in global scratch, the global-memory kernel), all slots
    forced into class >= min_cls, against the oracle and the reference's glue fixture."""
    monkeypatch.setenv("MC_BP_MIN_CLASS", str(min_cls))
    _check_dense(ctx)


@pytest.mark.parametrize("tier", [1, 2])
def test_voxel_kernels_match_oracle(ctx, monkeypatch, tier):
    """voxel_down_sample's kernels (the LDS tier every slot starts in; the larger LDS tier and the
    global-hash kernel it hands overflowing slots to), every slot forced onto the global kernel
    (tier 1) or the second LDS tier (tier 2), against the oracle and the reference's glue fixture."""
    monkeypatch.setenv("MC_VX_GLOBAL", str(tier))
    _check_dense(ctx)


@pytest.mark.parametrize("tier", [0, 2])
def test_high_resolution_voxel_tiers_match_oracle(ctx, monkeypatch, tier):
    """ScanNet++-resolution slots (thousands of voxels) through the first voxel tier and through the
    second (every slot forced there: its first 512 voxels' running sums in LDS, the rest in HBM)."""
    monkeypatch.setenv("MC_VX_GLOBAL", str(tier))
    from maskclustering_amd.synthetic_frames import make_frames_shape
    _check_against_oracle(ctx, make_frames_shape("tiny", seed=7, H=1440, W=1920, num_frames=1))


@pytest.mark.parametrize("ball_k", [7, 21, 32])
def test_ball_k_matches_oracle(ctx, ball_k):
    """ball_k other than the reference's 20: the query's 32-entry best list (ball_k > 20; five
    workgroups per CU) and the 20-entry one with fewer taken, against the CPU restatement."""
    from maskclustering_amd.synthetic_frames import make_frames_shape
    _check_against_oracle(ctx, make_frames_shape("tiny", seed=5, H=360, W=480, num_frames=3), ball_k=ball_k)


def test_high_resolution_frame_matches_oracle(ctx):
    """A ScanNet++-resolution frame (1920x1440): slots of tens of thousands of pixels and voxels of
    hundreds, against the CPU restatement."""
    from maskclustering_amd.synthetic_frames import make_frames_shape
    fr = make_frames_shape("tiny", seed=7, H=1440, W=1920, num_frames=1)
    _check_against_oracle(ctx, fr)


def test_odd_width_frames_match_oracle(ctx):
    """Frames whose width is not a multiple of 4 take the pixel kernels' one-pixel-per-lane path
    (the four-pixel loads need 4-pixel rows)."""
    from maskclustering_amd.synthetic_frames import make_frames_shape
    fr = make_frames_shape("tiny", seed=11, H=90, W=122, num_frames=4)
    _check_against_oracle(ctx, fr)


def test_misaligned_device_frames_match_aligned(ctx):
    """Device frames handed over at odd element offsets (a caller's tensor view): the pixel kernels'
    four-pixel vector loads need 16-byte depth / 4-byte seg alignment, so such frames take the
    one-pixel-per-lane path and give the same masks."""
    import torch
    from maskclustering_amd.synthetic_frames import make_frames_shape
    fr = make_frames_shape("tiny", seed=5, H=120, W=160, num_frames=3)
    want = _run(ctx, fr.scene_points, fr.depth, fr.seg, fr.intrinsics, fr.poses)
    dev = torch.device("cuda", 0)
    n = fr.depth.size
    dbuf = torch.zeros(n + 1, dtype=torch.float32, device=dev)
    sbuf = torch.zeros(n + 1, dtype=torch.uint8, device=dev)
    dbuf[1:] = torch.from_numpy(np.ascontiguousarray(fr.depth).reshape(-1)).to(dev)
    sbuf[1:] = torch.from_numpy(np.ascontiguousarray(fr.seg).reshape(-1)).to(dev)
    K = torch.from_numpy(np.ascontiguousarray(fr.intrinsics, np.float64)).to(dev)
    T = torch.from_numpy(np.ascontiguousarray(fr.poses, np.float64).reshape(-1, 16)).to(dev)
    d1, s1 = dbuf[1:], sbuf[1:]
    assert d1.data_ptr() % 16 != 0 and s1.data_ptr() % 4 != 0
    ctx.backproject(None, None, None, None, shape=fr.depth.shape,
                    device_ptrs=(d1.data_ptr(), s1.data_ptr(), K.data_ptr(), T.data_ptr()))
    torch.cuda.synchronize()
    for x, y in zip(want, ctx.bp_masks()):
        np.testing.assert_array_equal(x, y)


def _dense_inputs():
    from maskclustering_amd.synthetic_frames import make_frames_shape
    z = dict(np.load(os.path.join(GOLDEN, "s1_dense.npz")))
    fr = make_frames_shape("tiny", seed=5, H=360, W=480, num_frames=3)
    return [(z["in_scene"], z["in_depth"], z["in_seg"], z["in_intrinsics"], z["in_poses"]),
            (fr.scene_points, fr.depth, fr.seg, fr.intrinsics, fr.poses)]


@pytest.mark.parametrize("nbcap", [1, 8, 24, 63])
def test_list_overflow_paths_match_oracle(ctx, monkeypatch, nbcap):
    """The eps-neighbour lists are read only for counts <= nbcap; every longer list takes the cell-walk
    paths of the union, the border labels and the k-NN ring search.  Forcing the cap down sends most
    points (nbcap 1, 8) or the dense ones (24, 63) down those paths, in every size class: the results
    must still equal the oracle and the reference's glue fixture."""
    for min_cls in ("0", "2", "5"):
        monkeypatch.setenv("MC_BP_NBCAP", str(nbcap))
        monkeypatch.setenv("MC_BP_MIN_CLASS", min_cls)
        _check_dense(ctx)


def test_repeated_runs_identical(ctx):
    """Run-to-run determinism of the concurrent size classes (their lists are built with LDS-atomic
    slots, so any read of a slot before its store lands would vary between runs): the dense inputs
    against their references, then six more times each, every run bit-identical to the first."""
    _check_dense(ctx)
    for inp in _dense_inputs():
        want = _run(ctx, *inp)
        sa = ctx.bp_candidates()
        for _ in range(5):
            got = _run(ctx, *inp)
            np.testing.assert_array_equal(sa, ctx.bp_candidates())
            for x, y in zip(want, got):
                np.testing.assert_array_equal(x, y)


def test_diagnostics_build_invariants(ctx, tmp_path):
    """The in-kernel invariant checks on every driver run (they replace an in-process test that could
    only run with the diagnostics library loaded and was skipped otherwise): the -DMC_DBG_CHECK=1 build of the same
    source (maskclustering_amd/libmcgraph_dbg.so, built by __graft_entry__.build() behind the spill
    gate) in a worker process of its own (tests/dbg_invariants_worker.py): no check fails in any size
    class, lists full or capped, and its masks equal this (release) build's."""
    import subprocess
    import sys
    from maskclustering_amd import _native
    lib = os.path.join(os.path.dirname(_native.LIB_PATH), "libmcgraph_dbg.so")
    if not os.path.exists(lib):
        pytest.fail(f"{lib} missing: __graft_entry__.build() makes it")
    want = {}
    for i, inp in enumerate(_dense_inputs()):
        for k, x in enumerate(_run(ctx, *inp)):
            want[f"in{i}_{k}"] = np.asarray(x)
    path = tmp_path / "release_masks.npz"
    np.savez(path, **want)
    env = dict(os.environ, MCGRAPH_LIB=lib)
    env.pop("MC_BP_MIN_CLASS", None)
    env.pop("MC_BP_NBCAP", None)
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "dbg_invariants_worker.py"), str(path)],
                       env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]


def test_two_contexts_share_a_device_under_budgets():
    """Two live contexts on one device, each within its own HBM budget (mc_ctx_set_memory_budget;
    no MC_BP_BATCH_PIXELS): a budget that admits only a few frames per batch gives the same masks as
    the default one, whichever context runs, interleaved."""
    from maskclustering_amd import _native
    from maskclustering_amd.synthetic_frames import make_frames_shape
    fr = make_frames_shape("small", seed=2)
    F, H, W = fr.depth.shape
    a, b = _native.Context(0), _native.Context(0)
    b.set_memory_budget(224 * 3 * H * W)            # three frames per batch
    want = _run(a, fr.scene_points, fr.depth, fr.seg, fr.intrinsics, fr.poses)
    got = _run(b, fr.scene_points, fr.depth, fr.seg, fr.intrinsics, fr.poses)
    again = _run(a, fr.scene_points, fr.depth, fr.seg, fr.intrinsics, fr.poses)
    for x, y, z in zip(want, got, again):
        np.testing.assert_array_equal(x, y)
        np.testing.assert_array_equal(x, z)
    with pytest.raises(_native.McError):
        b.set_memory_budget(-1)


def test_denser_scene_after_sparse_one_stays_within_budget():
    """A stream of scenes on one context: the batches of a sparse scene are sized for its
    small mask-pixel share, so a denser scene after it overflows the per-batch arrays; the redo must
    take fewer frames per batch within the context's HBM budget (mc_ctx_set_memory_budget), not grow
    the arrays to the whole batch's mask pixels, and give the masks of a context without a budget."""
    from maskclustering_amd import _native
    from maskclustering_amd.synthetic_frames import make_frames_shape
    fr = make_frames_shape("small", seed=2)
    F, H, W = fr.depth.shape
    HW = H * W
    sparse = fr.seg.copy()
    for f in range(F):  # one mask per frame: the smallest id
        ids = np.unique(sparse[f])
        ids = ids[ids != 0]
        if len(ids):
            sparse[f][sparse[f] != ids[0]] = 0
    valid = (fr.depth > 0) & (fr.depth <= 20)
    dense_px = int(((fr.seg != 0) & valid).sum())
    sparse_px = int(((sparse != 0) & valid).sum())
    budget = max(int(0.5 * dense_px * 196), 250 * HW)
    assert dense_px * 196 > budget and sparse_px * 196 * 4 < budget   # the case the redo must bound
    ref = _native.Context(0)
    want_sparse = _run(ref, fr.scene_points, fr.depth, sparse, fr.intrinsics, fr.poses)
    want_dense = _run(ref, fr.scene_points, fr.depth, fr.seg, fr.intrinsics, fr.poses)
    ctx = _native.Context(0)
    ctx.set_memory_budget(budget)
    got_sparse = _run(ctx, fr.scene_points, fr.depth, sparse, fr.intrinsics, fr.poses)
    before = ctx.bp_batching()
    got_dense = _run(ctx, fr.scene_points, fr.depth, fr.seg, fr.intrinsics, fr.poses)
    after = ctx.bp_batching()
    for x, y in zip(want_sparse, got_sparse):
        np.testing.assert_array_equal(x, y)
    for x, y in zip(want_dense, got_dense):
        np.testing.assert_array_equal(x, y)
    assert after["redone"] > before["redone"], (before, after)
    assert after["frames_per_batch"] < F, after
    assert after["bytes_held"] <= budget + 196 * HW + 4 * F * HW + 196 * 2048, (budget, after)
