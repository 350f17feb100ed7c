"""Probe: a stream of C3 scenes on one GPU, sequential (S1 then S2-S6 per scene) against the scene
pipeline (frame_shard.ScenePipeline: S1 of scene k + 1 under the graph stages of scene k), per-scene
wall time and the objects of every scene compared between the two.

    python scripts/pipeline_probe.py [shape] [scenes]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from maskclustering_amd import _native  # noqa: E402
from maskclustering_amd.frame_shard import FrameShardedScene, ScenePipeline  # noqa: E402
from maskclustering_amd.pipeline import GraphRun  # noqa: E402
from maskclustering_amd.synthetic_frames import make_frames_shape  # noqa: E402

CFG = dict(mask_visible_threshold=0.3, undersegment_filter_threshold=0.3, view_consensus_threshold=0.9,
           contained_threshold=0.8)


def main():
    shape = sys.argv[1] if len(sys.argv) > 1 else "c3"
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    dev = torch.device("cuda", 0)
    fr = make_frames_shape(shape, seed=0, device="cuda:0", out="torch")
    F = fr.depth.shape[0]
    t_scene = torch.tensor(fr.scene_points, dtype=torch.float32, device=dev)
    K_t = torch.from_numpy(np.ascontiguousarray(fr.intrinsics)).to(dev)
    T_t = torch.from_numpy(np.ascontiguousarray(fr.poses.reshape(-1, 16))).to(dev)
    run = GraphRun(0)
    if os.environ.get("PROBE_PRIORITY"):  # the graph context on a high-priority stream
        hs = torch.cuda.Stream(device=dev, priority=-1)
        torch.cuda.set_stream(hs)
    run.ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    run.ctx.set_points(device_ptr=t_scene.data_ptr(), num_points=fr.num_points)
    s1 = _native.Context(0)
    s1.set_points(device_ptr=t_scene.data_ptr(), num_points=fr.num_points)
    free, _ = torch.cuda.mem_get_info()
    s1.set_memory_budget(int(free * 0.6))
    sh = FrameShardedScene(run, fr.num_points, F)
    pipe = ScenePipeline(sh, s1, fr.depth, fr.seg, K_t, T_t, _native.bp_params())

    def objects():
        ci = run.ctx.cluster_info()
        return run.ctx.objects(ci, F)

    # sequential: the same two contexts, one scene after the other
    def sequential(n):
        outs = []
        for _ in range(n):
            col, lab, off, pts = pipe._s1_scene()
            run.set_masks(fr.num_points, F, col, lab, off, pts_device_ptr=pts.data_ptr())
            sh.step(**CFG)
            outs.append(objects())
        return outs

    sequential(1)  # warm
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    seq = sequential(K)
    torch.cuda.synchronize()
    t_seq = (time.perf_counter() - t0) / K
    pip = []
    pipe.run(1, **CFG)  # warm
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pipe.run(K, on_scene=lambda k: pip.append(objects()), **CFG)
    torch.cuda.synchronize()
    t_pip = (time.perf_counter() - t0) / K
    same = all(all(np.array_equal(np.asarray(a[k]), np.asarray(b[k])) for k in a) for a, b in zip(seq, pip))
    print(f"{shape}: {K} scenes, sequential {t_seq * 1e3:.2f} ms/scene, pipelined {t_pip * 1e3:.2f} ms/scene, "
          f"objects identical: {same}", flush=True)
    if not same:
        sys.exit(1)


if __name__ == "__main__":
    main()
