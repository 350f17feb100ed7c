"""Frame-sharded S1 + all-gather + replicated S2-S6 against the
single-process run on the same frames: two ranks sharing cuda:0 (gloo carries the
gather; RCCL needs one GPU per rank, the bench's multi-GPU runs use it)."""
import numpy as np
import pytest

from shard_util import run_ranks

pytestmark = pytest.mark.gpu


def test_two_rank_frame_sharding_equals_single(tmp_path):
    from maskclustering_amd.pipeline import GraphRun
    from maskclustering_amd.synthetic_frames import make_frames_shape
    fr = make_frames_shape("small", seed=3)
    run = GraphRun(0)
    run.ctx.set_points(fr.scene_points.astype(np.float32))
    run.ctx.backproject(fr.depth, fr.seg, fr.intrinsics, fr.poses)
    col, lab, off, pts = run.ctx.bp_masks()
    run.set_masks(fr.num_points, fr.num_frames, col, lab, off, pts)
    run.step(0.3, 0.3, 0.9, 0.8)
    want = run.canonical()
    for out in run_ranks("e2e", 2, tmp_path):
        got = np.load(out)
        assert sorted(got.files) == sorted(want)
        for k in want:
            np.testing.assert_array_equal(got[k], np.asarray(want[k]), err_msg=k)
