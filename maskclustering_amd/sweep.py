"""Scene-parallel sweep over many scenes (BASELINE configs[4]: the 312-scene ScanNet val sweep), as the
reference's ``run.py:33-50`` runs it: one process per GPU, scene i on rank i mod N, each process
running ``main.py``'s path scene after scene, no collective on the data path.

Per scene (S1-S6 from frames resident in HBM): the scene's points (``mc_scene_set_points``, which
makes the next back-projection build the scene's ball-query grid), ``mc_backproject`` of every frame,
the masks as the graph input, ``mc_graph_build`` + ``mc_cluster_run``."""
from __future__ import annotations

import numpy as np


def scenes_of(rank: int, world: int, num_scenes: int) -> list[int]:
    """The scene numbers rank runs: i with i mod world == rank (run.py:33-50 hands scene lists to
    one process per GPU)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    return list(range(rank, int(num_scenes), world))


class SceneSweep:
    """One process's scenes on one device: ``run_scene`` per scene, the context reused across scenes
    (its S1 batches sized from the scenes before, within its HBM budget)."""

    def __init__(self, device: int, thresholds: dict, params=None, stream=None):
        from . import _native
        from .pipeline import GraphRun
        self.run = GraphRun(device)
        self.ctx = self.run.ctx
        if stream is not None:
            self.ctx.set_stream(stream)
        self.cfg = dict(thresholds)
        self.prm = params if params is not None else _native.bp_params()

    def run_scene(self, points, depth, seg, intrinsics, poses) -> int:
        """points float32 [P,3], depth f32 [F,H,W], seg u8 [F,H,W], intrinsics f64 [F,4], poses f64
        [F,16]: contiguous torch tensors on the device.  Returns the scene's object count; the
        context holds the scene's full result (GraphRun.canonical, the getters)."""
        for t in (points, depth, seg, intrinsics, poses):
            if t.device.type != "cuda" or not t.is_contiguous():
                raise ValueError("scene inputs must be contiguous device tensors")
        F, H, W = depth.shape
        self.ctx.set_points(device_ptr=points.data_ptr(), num_points=len(points))
        self.ctx.backproject(None, None, None, None, self.prm, shape=(F, H, W),
                             device_ptrs=(depth.data_ptr(), seg.data_ptr(), intrinsics.data_ptr(), poses.data_ptr()))
        col, lab, _ = self.ctx.bp_mask_index()
        self.run.P, self.run.F = len(points), F
        self.run.mask_col, self.run.mask_label = np.asarray(col), np.asarray(lab)
        self.ctx.use_backprojection()
        self.run.step(**self.cfg)
        return int(self.ctx.cluster_info().num_objects)
