"""One rank's share of an N-GPU frame-sharded C3 scene, measured on one GPU.

The bench's default at N ranks: each rank back-projects its frame slice (S1), the mask CSRs are
all-gathered, and every rank runs the graph stages on the whole scene's masks; with the scene
pipeline (frame_shard.ScenePipeline) the graph stages of scene k run beside S1 of scene k + 1.
Without N GPUs this script runs what one rank's device does: S1 of the rank's cost-balanced slice
in a producer thread on its own context, and the graph stages over the WHOLE scene's masks (made
once up front, handed to the graph context as the gather would) in the calling thread, scene after
scene.  The graph stages run unsharded here (the bench shards S3 / S4 / S6 level 0 N ways): an
upper bound on the rank's graph work.  The gather of the mask CSRs (issued by the consumer thread,
under the producer's S1) is modelled in the consumer thread, per scene, before the graph stages: a device copy of the rank's share of the point ids (the bytes it sends; the owner
receives N - 1 such shares, one per peer link, in parallel) plus a host wait of those bytes over one
xGMI link at XGMI_LINK_GBS (64 GB/s, a conservative one-direction rate of a 153 GB/s link).  Prints
one JSON line per N.

    python scripts/rank_proxy.py [shape] [scenes] [N ...]
"""
import json
import os
import queue
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from maskclustering_amd import _native  # noqa: E402
from maskclustering_amd.frame_shard import FrameShardedScene, balanced_frame_slices, frame_costs  # noqa: E402
from maskclustering_amd.pipeline import GraphRun  # noqa: E402
from maskclustering_amd.synthetic_frames import make_frames_shape  # noqa: E402

from maskclustering_amd.dataset_configs import shape_thresholds  # noqa: E402

XGMI_LINK_GBS = float(os.environ.get("MC_PROXY_LINK_GBS", "64"))


def main():
    shape = sys.argv[1] if len(sys.argv) > 1 else "c3"
    CFG = shape_thresholds(shape)[1]
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    Ns = [1] + [n for n in ([int(x) for x in sys.argv[3:]] or [8]) if n != 1]
    dev = torch.device("cuda", 0)
    t0 = time.perf_counter()
    fr = make_frames_shape(shape, seed=0, device="cuda:0", out="torch")
    F = fr.depth.shape[0]
    print(f"{shape}: {F} frames rendered in {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
    t_scene = torch.tensor(fr.scene_points, dtype=torch.float32, device=dev)
    K_t = torch.from_numpy(np.ascontiguousarray(fr.intrinsics)).to(dev)
    T_t = torch.from_numpy(np.ascontiguousarray(fr.poses.reshape(-1, 16))).to(dev)
    prm = _native.bp_params()
    run = GraphRun(0)
    run.ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    run.ctx.set_points(device_ptr=t_scene.data_ptr(), num_points=fr.num_points)
    s1 = _native.Context(0)
    s1.set_points(device_ptr=t_scene.data_ptr(), num_points=fr.num_points)
    free, _ = torch.cuda.mem_get_info()
    s1.set_memory_budget(int(free * 0.5))
    sh = FrameShardedScene(run, fr.num_points, F)

    s1b = None  # a second S1 context (two producers: one scene's kernel tails filled by the next's)
    if os.environ.get("MC_PROXY_TWO_PRODUCERS", "0") != "0":  # (the bench's default is one producer)
        s1b = _native.Context(0)
        s1b.set_points(device_ptr=t_scene.data_ptr(), num_points=fr.num_points)
        s1b.set_memory_budget(int(free * 0.3))

    def s1_masks(lo, hi, s1=s1):
        s1.set_points(device_ptr=t_scene.data_ptr(), num_points=fr.num_points)  # per scene, as the bench
        s1.backproject(None, None, None, None, prm, shape=(hi - lo, fr.depth.shape[1], fr.depth.shape[2]),
                       device_ptrs=(fr.depth[lo:hi].data_ptr(), fr.seg[lo:hi].data_ptr(), K_t[lo:hi].data_ptr(),
                                    T_t[lo:hi].data_ptr()))
        col, lab, off = s1.bp_mask_index()
        pts = torch.empty(max(int(off[-1]), 1), dtype=torch.int32, device=dev)
        s1.bp_points_to_device(pts.data_ptr())
        s1.synchronize()
        return col, lab, off, pts

    full = s1_masks(0, F)  # the gathered masks every rank's graph stages read
    nnz_all = int(full[2][-1])
    scratch = torch.empty(max(nnz_all, 1), dtype=torch.int32, device=dev)

    def gather_model(N):
        """the rank's share of one scene's point-id gather: its slice's ids copied on the device, and
        the host wait of those bytes over one link (the owner's N - 1 incoming shares arrive in parallel)"""
        if N == 1:
            return 0.0
        share = max(1, nnz_all // N)
        t = time.perf_counter()
        scratch[:share].copy_(full[3][:share])
        torch.cuda.current_stream().synchronize()
        time.sleep(4.0 * share / (XGMI_LINK_GBS * 1e9))
        return time.perf_counter() - t

    def graph():
        col, lab, off, pts = full
        run.set_masks(fr.num_points, F, col, lab, off, pts_device_ptr=pts.data_ptr())
        sh.step(**CFG)
        return run.ctx.cluster_info().num_objects

    def timed(fn, n):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / n * 1e3

    objects = graph()
    g_ms = timed(graph, K)
    one_ms = timed(lambda: (s1_masks(0, F), graph()), max(2, K // 2))
    base_pipe = None
    costs = frame_costs(fr.depth, fr.seg, K_t).cpu().numpy()
    for N in Ns:
        print(f"N = {N}", file=sys.stderr, flush=True)
        slices = balanced_frame_slices(costs, N)
        s1_ms = [timed(lambda: s1_masks(lo, hi), max(2, K // 2)) for lo, hi in slices]
        r = int(np.argmax(s1_ms))
        lo, hi = slices[r]

        def pipelined(n, every=1):
            q: queue.Queue = queue.Queue(maxsize=1)

            def produce():
                try:
                    for _ in range(n):
                        q.put(s1_masks(lo, hi))
                except BaseException as e:  # handed to the consumer, which raises it
                    q.put(e)

            th = threading.Thread(target=produce, daemon=True)
            th.start()
            for k in range(n):
                if isinstance(q.get(), BaseException):
                    raise RuntimeError("S1 producer failed")
                gather_model(N)
                if k % every == 0:  # scene-owner mode: this rank's scenes only
                    graph()
            th.join()

        def timed_pipe(n, every=1):
            pipelined(1)
            torch.cuda.synchronize()
            t = time.perf_counter()
            pipelined(n, every)
            torch.cuda.synchronize()
            return (time.perf_counter() - t) / n * 1e3

        pipe_ms = timed_pipe(K)
        base_pipe = base_pipe or pipe_ms
        # scene-owner graph stages (the bench default at N > 1): the rank runs them for every N-th scene;
        # over N * ceil(K / N) scenes so that the share is exact
        Ko = N * max(1, -(-K // N))
        own_ms = timed_pipe(Ko, N)

        def pipelined2(n, every):  # two producers on two S1 contexts, scenes alternating, taken in order
            qs = [queue.Queue(maxsize=1), queue.Queue(maxsize=1)]

            def produce(i, ctx):
                for _ in range(i, n, 2):
                    qs[i].put(s1_masks(lo, hi, ctx))

            ths = [threading.Thread(target=produce, args=(i, c), daemon=True) for i, c in enumerate((s1, s1b))]
            for th in ths:
                th.start()
            for k in range(n):
                qs[k % 2].get()
                gather_model(N)
                if k % every == 0:
                    graph()
            for th in ths:
                th.join()

        own2_ms = None
        if s1b is not None and N > 1:  # (a whole C3 scene twice does not fit beside the first context's arrays)
            pipelined2(2, N)
            torch.cuda.synchronize()
            t = time.perf_counter()
            pipelined2(Ko, N)
            torch.cuda.synchronize()
            own2_ms = (time.perf_counter() - t) / Ko * 1e3
        print(json.dumps({
            "shape": shape, "N": N, "objects": int(objects), "scenes": K,
            "one_gpu_sequential_ms": round(one_ms, 3),
            "graph_stages_full_scene_ms": round(g_ms, 3),
            "s1_slice_ms": [round(x, 3) for x in s1_ms], "slowest_slice": [int(lo), int(hi)],
            "rank_pipelined_ms": round(pipe_ms, 3),
            "rank_sequential_ms": round(s1_ms[r] + g_ms, 3),
            "projected_speedup": round(base_pipe / pipe_ms, 2),
            "rank_pipelined_scene_owner_ms": round(own_ms, 3), "scene_owner_scenes": Ko,
            "projected_speedup_scene_owner": round(base_pipe / own_ms, 2),
            "rank_two_producers_scene_owner_ms": own2_ms and round(own2_ms, 3),
            "gather_model_ms": round(1e3 * gather_model(N), 3), "point_ids_per_scene": nnz_all,
            "xgmi_link_gbs": XGMI_LINK_GBS,
            "projected_speedup_two_producers": own2_ms and round(base_pipe / own2_ms, 2),
            "note": "rank_pipelined_ms: S1 of the slowest slice beside the unsharded graph stages of the previous "
                    "scene; projected_speedup: the N = 1 line's rank_pipelined_ms over this one; every scene's share "
                    "of the point-id gather is modelled in the consumer thread (gather_model_ms: a device copy of "
                    "the rank's share + its bytes over one xGMI link); scene_owner: the graph stages of every N-th "
                    "scene only"}),
              flush=True)


if __name__ == "__main__":
    main()
