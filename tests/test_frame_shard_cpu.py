"""Frame sharding on the CPU: slice arithmetic, the all-gather of per-rank mask
CSRs, and the row-block sharded S2-S6 (maskclustering_amd.graph_shard.ShardedGraph: S3 row blocks,
S4 histogram shares summed, S6 level-0 union-find forests united) over gloo at world sizes 1-8 (a
rank with no frames included), against the single-process result, and the reference's container
orders from the sharded run's gathered edges.  The per-rank compute is the sparse oracle behind the same
exchange API as the HIP library (tests/oracle_shard_ctx.py); the GPU twin is
tests/test_gpu_frame_shard.py."""
import numpy as np
import pytest

from shard_util import run_ranks


def test_frame_slices_cover_frames_in_order():
    from maskclustering_amd.frame_shard import frame_slice
    for F in (0, 1, 2, 7, 250, 1501):
        for world in (1, 2, 3, 4, 8, 16):
            sl = [frame_slice(F, world, r) for r in range(world)]
            assert sl[0][0] == 0 and sl[-1][1] == F
            assert all(a[1] == b[0] for a, b in zip(sl, sl[1:]))
            sizes = [hi - lo for lo, hi in sl]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        frame_slice(10, 2, 2)


def test_balanced_slices_split_cost_evenly():
    from maskclustering_amd.frame_shard import balanced_frame_slices, frame_slice
    rng = np.random.default_rng(0)
    for F in (1, 2, 7, 250, 1500):
        for world in (1, 2, 3, 8, 16):
            for kind in ("flat", "skew", "random", "zeros", "spike"):
                c = {"flat": np.ones(F), "skew": np.where(np.arange(F) < max(1, F // 4), 50.0, 1.0),
                     "random": rng.gamma(2.0, 1.0, F), "zeros": np.zeros(F),
                     "spike": np.eye(1, F, F // 2).ravel() * 1e6 + 1.0}[kind]
                sl = balanced_frame_slices(c, world)
                assert len(sl) == world and sl[0][0] == 0 and sl[-1][1] == F
                assert all(a[1] == b[0] and a[0] <= a[1] for a, b in zip(sl, sl[1:]))
                assert [frame_slice(F, world, r, costs=c) for r in range(world)] == sl
                if kind == "zeros":
                    assert sl == [frame_slice(F, world, r) for r in range(world)]
                    continue
                # every slice within one frame's cost of the even share
                share = c.sum() / world
                for lo, hi in sl:
                    assert c[lo:hi].sum() <= share + c.max() + 1e-9
    with pytest.raises(ValueError):
        balanced_frame_slices([1.0, -1.0], 2)


def test_frame_costs_count_mask_pixels_and_footprints():
    import torch
    from maskclustering_amd.frame_shard import frame_costs
    depth = torch.zeros(3, 4, 6)
    seg = torch.zeros(3, 4, 6, dtype=torch.uint8)
    depth[0] = 2.0
    seg[0, :2] = 5                       # 12 mask pixels at 2 m
    depth[1, :, :3] = 30.0               # beyond DEPTH_TRUNC: no mask pixels
    seg[1] = 1
    depth[2] = 1.0
    seg[2, 0, 0] = 7                     # one pixel
    K = np.tile([100.0, 100.0, 3.0, 2.0], (3, 1))
    c = frame_costs(depth, seg, K, pixel_weight=1.0, voxel_weight=10.0, frame_weight=0.0).numpy()
    foot = lambda d: min(1.0, d * d / (100.0 * 100.0 * 1e-4))  # noqa: E731
    np.testing.assert_allclose(c, [12 * (1 + 10 * foot(2.0)), 0.0, 1 + 10 * foot(1.0)], rtol=1e-6)


@pytest.mark.parametrize("world", [3, 4, 8])
def test_skewed_scene_balanced_slices_equal_single_process(tmp_path, world):
    """A scene whose masks crowd into the first quarter of the frames: the cost-balanced slices
    differ from the equal-count ones, and every rank still ends with the single-process result."""
    from maskclustering_amd.synthetic import make_shape
    from oracle import oracle
    from shard_worker import skewed
    s = skewed(make_shape("c1", seed=1))
    want = oracle.run_sparse(s.num_points, s.num_frames, s.mask_col, s.mask_label, s.mask_off, s.mask_pts,
                             **KW["scannet"])
    lens = np.diff(s.mask_off).astype(np.float64)
    costs = np.bincount(s.mask_col, weights=lens, minlength=s.num_frames)
    for out in run_ranks("skew:c1:1", world, tmp_path):
        got = np.load(out)
        np.testing.assert_array_equal(got["costs"], costs)
        sl = [tuple(x) for x in got["slices"]]
        assert sl[0][1] < s.num_frames // world  # the crowded first slice is short
        share = [costs[lo:hi].sum() for lo, hi in sl]
        assert max(share) <= costs.sum() / world + costs.max()
        for k in want:
            np.testing.assert_array_equal(got[k], np.asarray(want[k]), err_msg=k)


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_gather_equals_global_mask_list(tmp_path, world):
    from maskclustering_amd.synthetic import make_shape
    s = make_shape("tiny", seed=4)
    for out in run_ranks("gather", world, tmp_path):
        z = np.load(out)
        np.testing.assert_array_equal(z["col"], s.mask_col)
        np.testing.assert_array_equal(z["label"], s.mask_label)
        np.testing.assert_array_equal(z["off"], s.mask_off)
        np.testing.assert_array_equal(z["pts"], s.mask_pts)


@pytest.mark.parametrize("mode", ["gather_dst", "gather_dst_nogather"])
@pytest.mark.parametrize("world", [2, 3])
def test_gather_to_one_rank(tmp_path, world, mode):
    """gather_masks(dst=last rank): every rank gets the global mask index, only dst the point ids, by
    dist.gather or (a backend without gather, chosen alike on every rank) by the all-gather."""
    from maskclustering_amd.synthetic import make_shape
    s = make_shape("tiny", seed=4)
    for r, out in enumerate(run_ranks(mode, world, tmp_path)):
        z = np.load(out)
        np.testing.assert_array_equal(z["col"], s.mask_col)
        np.testing.assert_array_equal(z["label"], s.mask_label)
        np.testing.assert_array_equal(z["off"], s.mask_off)
        assert bool(z["has_pts"][0]) == (r == world - 1)
        if r == world - 1:
            np.testing.assert_array_equal(z["pts"], s.mask_pts)


def test_scene_pipeline_producer_and_consumer_errors_do_not_hang():
    """The consumer raises (on_scene) while a producer holds an exception for a full queue: run()
    re-raises the consumer's error promptly instead of waiting on the producer forever."""
    import threading

    import torch
    from maskclustering_amd.frame_shard import FrameShardedScene, ScenePipeline
    failed = threading.Event()

    class S1Ctx:
        n = 0

        def backproject(self, *a, **kw):
            S1Ctx.n += 1
            if S1Ctx.n == 3:
                failed.set()
                raise RuntimeError("producer failure")

        def bp_mask_index(self):
            return np.zeros(1, np.int32), np.ones(1, np.int32), np.array([0, 2], np.int64)

        def bp_points_to_device(self, dst):
            pass

        def synchronize(self):
            pass

        def stream(self):
            return 0

    class Run:
        ctx = None

        def set_masks(self, *a, **kw):
            pass

        def step(self, *a):
            pass

    sh = FrameShardedScene(Run(), 10, 1, shard_graph=False)
    z = torch.zeros((1, 1, 1))

    def on_scene(k):
        failed.wait(10)  # the producer's error is pending behind the queued scene 1
        raise ValueError("consumer failure")

    pipe = ScenePipeline(sh, S1Ctx(), z, z.to(torch.uint8), torch.zeros((1, 4), dtype=torch.float64),
                         torch.zeros((1, 16), dtype=torch.float64))
    err = []

    def go():
        try:
            pipe.run(5, on_scene=on_scene, **KW["scannet"])
        except BaseException as e:  # noqa: BLE001
            err.append(e)

    th = threading.Thread(target=go, daemon=True)
    th.start()
    th.join(20)
    assert not th.is_alive(), "ScenePipeline.run hung on the producer's pending exception"
    assert len(err) == 1 and isinstance(err[0], ValueError)


KW = {"scannet": dict(mask_visible_threshold=0.3, undersegment_filter_threshold=0.3, view_consensus_threshold=0.9,
                      contained_threshold=0.8),
      "scannetpp": dict(mask_visible_threshold=0.4, undersegment_filter_threshold=0.2, view_consensus_threshold=1,
                        contained_threshold=0.9)}


@pytest.mark.parametrize("world,shape,seed,cfg", [(1, "tiny", 4, "scannet"), (2, "tiny", 4, "scannet"),
                                                  (3, "tiny", 5, "scannetpp"), (2, "c1", 1, "scannet"),
                                                  (3, "c1", 2, "scannet"), (4, "c1", 3, "scannet"),
                                                  (8, "c1", 1, "scannetpp"), (8, "few", 0, "scannet")])
def test_sharded_graph_equals_single_process(tmp_path, world, shape, seed, cfg):
    """Every rank ends with exactly the single-process S2-S6 outputs (every stage, canonical form)."""
    from maskclustering_amd.synthetic import make_shape
    from oracle import oracle
    s = make_shape(shape, seed=seed)
    want = oracle.run_sparse(s.num_points, s.num_frames, s.mask_col, s.mask_label, s.mask_off, s.mask_pts, **KW[cfg])
    assert int(want["num_iters"]) > 1
    for out in run_ranks(f"graph:{shape}:{seed}:{cfg}", world, tmp_path):
        got = np.load(out)
        assert sorted(got.files) == sorted(want)
        for k in want:
            np.testing.assert_array_equal(got[k], np.asarray(want[k]), err_msg=k)


@pytest.mark.parametrize("world,shape,seed,cfg", [(2, "c1", 1, "scannet"), (4, "tiny", 5, "scannetpp"),
                                                  (8, "few", 0, "scannet")])
def test_sharded_reference_orders_equal_single_process(tmp_path, world, shape, seed, cfg):
    """The reference's container orders (mc_setorder_replay) from a sharded run, whose iteration-0
    edges are gathered from the ranks' pair rows, equal those of the single-process run's edges."""
    from maskclustering_amd import _native
    from maskclustering_amd.synthetic import make_shape
    from oracle import oracle
    s = make_shape(shape, seed=seed)
    want = oracle.run_sparse(s.num_points, s.num_frames, s.mask_col, s.mask_label, s.mask_off, s.mask_pts,
                             edge_cap=1 << 20, **KW[cfg])
    T = int(want["num_iters"])
    assert T > 1
    tt, aa, bb = want["edges"]
    node0 = want["node0_g"]            # every input mask is global in these scenes
    assert len(want["gl_col"]) == len(s.mask_col)
    po = np.zeros(len(node0) + 1, np.int64)
    np.cumsum(np.diff(s.mask_off)[node0], out=po[1:])
    seqs = np.concatenate([s.mask_points(g) for g in node0]).astype(np.int32)
    ref = _native.setorder_replay(want["level_sizes"][:T], np.searchsorted(tt, np.arange(T + 1)), aa, bb, po, seqs,
                                  labels=True)
    for out in run_ranks(f"orders:{shape}:{seed}:{cfg}", world, tmp_path):
        got = np.load(out)
        for k in ref:
            np.testing.assert_array_equal(got[k], ref[k], err_msg=k)


def test_sharded_edges_overflow_raises_on_every_rank(tmp_path):
    """Rank 0's edge capture overflows (capacity 2): edges() must raise on every rank before any
    exchange (the other ranks would otherwise wait in the all-gather rank 0 never joins), and with the
    capacity grown every rank gets the same gathered edges."""
    outs = [np.load(o) for o in run_ranks("overflow:c1:1:scannet", 2, tmp_path)]
    assert [int(o["raised"][0]) for o in outs] == [1, 1]
    for k in ("tt", "aa", "bb"):
        np.testing.assert_array_equal(outs[0][k], outs[1][k])
    assert len(outs[0]["tt"]) > 2


@pytest.mark.parametrize("world,shape,seed,cfg", [(1, "c1", 1, "scannet"), (2, "c1", 1, "scannet"),
                                                  (4, "tiny", 5, "scannetpp")])
def test_scene_pipeline_equals_single_process(tmp_path, world, shape, seed, cfg):
    """The scene pipeline (S1 in a producer thread, gather + sharded S2-S6 in the calling thread, three
    scenes): every scene on every rank ends with exactly the single-process S2-S6 outputs, and S1 ran
    once per scene."""
    from maskclustering_amd.synthetic import make_shape
    from oracle import oracle
    s = make_shape(shape, seed=seed)
    want = oracle.run_sparse(s.num_points, s.num_frames, s.mask_col, s.mask_label, s.mask_off, s.mask_pts, **KW[cfg])
    for out in run_ranks(f"pipeline:{shape}:{seed}:{cfg}", world, tmp_path):
        got = np.load(out)
        assert int(got["s1_calls"][0]) == 3
        for k in range(3):
            for name in want:
                np.testing.assert_array_equal(got[f"{k}/{name}"], np.asarray(want[name]), err_msg=f"scene {k} {name}")


@pytest.mark.parametrize("world,shape,seed,cfg,mode", [(2, "c1", 1, "scannet", "owner"), (3, "tiny", 5, "scannetpp", "owner"),
                                                       (4, "c1", 2, "scannet", "owner"), (2, "c1", 1, "scannet", "owner2"),
                                                       (3, "c1", 2, "scannet", "owner2")])
def test_scene_owner_pipeline_equals_single_process(tmp_path, world, shape, seed, cfg, mode):
    """The scene-owner pipeline (every rank back-projects its slice of every scene; scene k's masks
    are gathered to rank k mod world alone, which runs S2-S6 unsharded): each scene is clustered by
    exactly one rank, its owner, with exactly the single-process outputs, and S1 ran on every rank
    for every scene.  Two run() calls, the first with one scene (the bench's warmup), the second
    starting at owner 1.  owner2: two S1 producers on two contexts, scenes alternating."""
    from maskclustering_amd.synthetic import make_shape
    from oracle import oracle
    s = make_shape(shape, seed=seed)
    want = oracle.run_sparse(s.num_points, s.num_frames, s.mask_col, s.mask_label, s.mask_off, s.mask_pts, **KW[cfg])
    nsc = 2 * world + 1
    seen = []
    for r, out in enumerate(run_ranks(f"{mode}:{shape}:{seed}:{cfg}", world, tmp_path)):
        got = np.load(out)
        assert int(got["s1_calls"][0]) == nsc
        owned = [int(k) for k in got["owned"]]
        assert owned == [k for k in range(nsc) if k % world == r]
        seen += owned
        for k in owned:
            for name in want:
                np.testing.assert_array_equal(got[f"{k}/{name}"], np.asarray(want[name]), err_msg=f"scene {k} {name}")
    assert sorted(seen) == list(range(nsc))


def test_sweep_scene_assignment_covers_each_scene_once():
    """run.py:33-50's split of the scene list over one process per GPU: scene i on rank i mod N."""
    from maskclustering_amd.sweep import scenes_of
    for world in (1, 2, 3, 8):
        got = sorted(i for r in range(world) for i in scenes_of(r, world, 312))
        assert got == list(range(312))
        assert all(i % world == r for r in range(world) for i in scenes_of(r, world, 312))
    with pytest.raises(ValueError):
        scenes_of(2, 2, 10)
