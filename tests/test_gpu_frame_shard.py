"""Frame-sharded S1 + all-gather + row-block sharded S2-S6 (SURVEY.md §8(e),
maskclustering_amd/graph_shard.py) through the HIP library against the single-process run on
the same input: two and three ranks sharing cuda:0 (gloo carries the exchanges; RCCL needs one
GPU per rank, the bench's multi-GPU runs use it)."""
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


@pytest.mark.parametrize("world,shape,seed", [(2, "c1", 1), (3, "c1", 2)])
def test_sharded_graph_stages_equal_single(tmp_path, world, shape, seed):
    """S3 row blocks, S4 histogram shares and S6 level-0 forests over the ranks give every rank the
    single-GPU result, every stage compared."""
    from maskclustering_amd.pipeline import GraphRun
    from maskclustering_amd.synthetic import make_shape
    s = make_shape(shape, seed=seed)
    run = GraphRun(0)
    run.set_scene(s)
    run.step(0.3, 0.3, 0.9, 0.8)
    want = run.canonical(dense=False)
    assert int(want["num_iters"]) > 1
    for out in run_ranks(f"gpugraph:{shape}:{seed}", world, tmp_path):
        got = np.load(out)
        assert sorted(got.files) == sorted(want)
        for k in want:
            np.testing.assert_array_equal(got[k], np.asarray(want[k]), err_msg=k)


def test_native_rccl_exchanges_equal_single():
    """mc_ctx_comm_init (the library's own RCCL communicator): with a one-rank
    communicator the sharded flow runs every exchange through RCCL inside mc_graph_build /
    mc_cluster_run (all-gather / all-reduce of one block: identities), and every stage equals the
    single-process run; detaching restores the plain path."""
    from maskclustering_amd.graph_shard import ShardedGraph
    from maskclustering_amd.pipeline import GraphRun
    from maskclustering_amd.synthetic import make_shape
    s = make_shape("c1", seed=1)
    run = GraphRun(0)
    run.set_scene(s)
    run.step(0.3, 0.3, 0.9, 0.8)
    want = run.canonical(dense=False)
    run2 = GraphRun(0)
    run2.set_scene(s)
    sh = ShardedGraph(run2, native_comm=True)
    sh.step(0.3, 0.3, 0.9, 0.8)
    assert run2.ctx.shard_pending() == 0
    got = run2.canonical(dense=False)
    for k in want:
        np.testing.assert_array_equal(np.asarray(got[k]), np.asarray(want[k]), err_msg=k)
    run2.ctx.attach_comm(None)
    run2.step(0.3, 0.3, 0.9, 0.8)
    got = run2.canonical(dense=False)
    for k in want:
        np.testing.assert_array_equal(np.asarray(got[k]), np.asarray(want[k]), err_msg=k)
