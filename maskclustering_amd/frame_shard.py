"""Frame-sharded scenes over ranks (BASELINE north_star).

One process per GPU.  Rank r owns the contiguous frame slice ``frame_slice(F, world, r)``
and runs S1 (``utils/mask_backprojection.py:70-151``, per frame and independent across
frames) on its own GPU, so every frame's masks are exactly the single-GPU ones.  The
per-rank mask CSRs are then all-gathered in rank order.  Slices are contiguous and
ascending, so the concatenation is the reference's global mask order (frames ascending,
ids ascending: ``graph/construction.py:46-60``).  The graph stages then run row-block
sharded (``graph_shard.ShardedGraph``: S3 rows, S4 histogram tiles and S6's first N0 x N0
pair evaluation split over the ranks, exchanged as row blocks, one summed histogram and
union-find forests); every process ends with the full result, as the reference's
per-process callers expect (``main.py:17-19``).

Exchanges per scene: the mask lists (C2 ≈ 15 MB of point ids, C3 ≈ 105 MB), the S3 rows
(C3 ≈ 13 MB), the histogram (8·(F+1) B) and the forests (4·N0 B per rank).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def frame_slice(num_frames: int, world: int, rank: int) -> tuple[int, int]:
    """[lo, hi) of the frames rank owns: contiguous, sizes differ by at most one."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    base, extra = divmod(int(num_frames), world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def _comm_device(group, like: torch.device) -> torch.device:
    """Tensors for the collective: device tensors under RCCL ("nccl"), host tensors under gloo."""
    return like if dist.get_backend(group) == "nccl" else torch.device("cpu")


def gather_masks(mask_col, mask_label, mask_off, mask_pts: torch.Tensor, frame_lo: int, group=None):
    """All-gather per-rank mask CSRs into the global one.

    mask_col / mask_label / mask_off: this rank's masks (numpy; mask_col relative to
    frame_lo); mask_pts: int32 tensor of their point ids (any device).
    Returns (mask_col, mask_label, mask_off int64) as numpy and the global point ids as an
    int32 tensor on mask_pts' device.
    """
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    out_dev = mask_pts.device
    col = np.asarray(mask_col, np.int32) + np.int32(frame_lo)
    lab = np.asarray(mask_label, np.int32)
    off = np.asarray(mask_off, np.int64)
    M = len(col)
    nnz = int(off[M]) if M else 0
    if len(off) != M + 1 or len(lab) != M or mask_pts.numel() < nnz:
        raise ValueError("inconsistent mask CSR")
    if world == 1:
        return col, lab, off.copy(), mask_pts[:nnz].clone()
    dev = _comm_device(group, out_dev)
    sizes = torch.tensor([M, nnz], dtype=torch.int64, device=dev)
    all_sizes = [torch.empty_like(sizes) for _ in range(world)]
    dist.all_gather(all_sizes, sizes, group=group)
    Ms = [int(x[0]) for x in all_sizes]
    Ns = [int(x[1]) for x in all_sizes]
    mmax, nmax = max(1, max(Ms)), max(1, max(Ns))
    meta = np.zeros((3, mmax), np.int32)
    meta[0, :M], meta[1, :M], meta[2, :M] = col, lab, np.diff(off)
    meta_t = torch.from_numpy(meta).to(dev)
    metas = [torch.empty_like(meta_t) for _ in range(world)]
    dist.all_gather(metas, meta_t, group=group)
    buf = torch.zeros(nmax, dtype=torch.int32, device=dev)
    buf[:nnz] = mask_pts[:nnz].to(dev)
    bufs = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(bufs, buf, group=group)
    metas = [m.cpu().numpy() for m in metas]
    g_col = np.concatenate([m[0, :k] for m, k in zip(metas, Ms)]).astype(np.int32)
    g_lab = np.concatenate([m[1, :k] for m, k in zip(metas, Ms)]).astype(np.int32)
    g_len = np.concatenate([m[2, :k] for m, k in zip(metas, Ms)]).astype(np.int64)
    g_off = np.zeros(len(g_len) + 1, np.int64)
    np.cumsum(g_len, out=g_off[1:])
    g_pts = torch.cat([b[:n] for b, n in zip(bufs, Ns)]).to(out_dev)
    return g_col, g_lab, g_off, g_pts


class FrameShardedScene:
    """S1 on this rank's frames, all-gather, then the replicated graph path.

    ``run`` is this rank's :class:`maskclustering_amd.pipeline.GraphRun` (its context holds
    the scene points: ``ctx.set_points``).  Inputs of :meth:`backproject` are this rank's
    frame slice, resident on its GPU.
    """

    def __init__(self, run, num_points: int, num_frames: int, group=None, shard_graph: bool = True):
        from .graph_shard import ShardedGraph
        self.run = run
        self.ctx = run.ctx
        self.P, self.F = int(num_points), int(num_frames)
        self.group = group
        on = dist.is_initialized()
        self.rank = dist.get_rank(group) if on else 0
        self.world = dist.get_world_size(group) if on else 1
        self.lo, self.hi = frame_slice(self.F, self.world, self.rank)
        self._pts = None  # global point ids (kept alive until the graph input copy is done)
        # the graph stages row-block sharded over the same ranks (shard_graph=False: replicated)
        self.graph = ShardedGraph(run, group) if shard_graph else None

    @property
    def pts(self) -> torch.Tensor:
        """The global mask point ids (int32); a single-process run reads them from the context."""
        if self._pts is None and self.world == 1 and getattr(self, "mask_index", None) is not None:
            self._pts = torch.from_numpy(np.ascontiguousarray(self.ctx.bp_masks()[3]))
        return self._pts

    @pts.setter
    def pts(self, v):
        self._pts = v

    def set_local_masks(self, mask_col, mask_label, mask_off, mask_pts: torch.Tensor):
        """This rank's frames' masks (mask_col relative to the slice) as the S1 output would
        leave them (the G variant's input): all-gathered into the graph input."""
        g_col, g_lab, g_off, self.pts = gather_masks(mask_col, mask_label, mask_off, mask_pts, self.lo, self.group)
        self.mask_index = (g_col, g_lab, g_off)
        if self.pts.device.type == "cuda":
            torch.cuda.current_stream(self.pts.device).synchronize()
            self.run.set_masks(self.P, self.F, g_col, g_lab, g_off, pts_device_ptr=self.pts.data_ptr())
        else:
            self.run.set_masks(self.P, self.F, g_col, g_lab, g_off, self.pts.numpy())
        return g_col, g_lab, g_off

    def backproject(self, depth: torch.Tensor, seg: torch.Tensor, intrinsics: torch.Tensor,
                    poses: torch.Tensor, params=None):
        """depth f32 [n,H,W], seg u8 [n,H,W], intrinsics f64 [n,4], poses f64 [n,16] on this
        rank's GPU, n = hi - lo.  Leaves the global masks as the graph input."""
        n = self.hi - self.lo
        if depth.shape[0] != n or seg.shape != depth.shape or intrinsics.shape[0] != n or poses.shape[0] != n:
            raise ValueError(f"rank {self.rank} owns {n} frames [{self.lo}, {self.hi})")
        for t, dt in ((depth, torch.float32), (seg, torch.uint8), (intrinsics, torch.float64),
                      (poses, torch.float64)):
            if t.dtype != dt or not t.is_contiguous() or t.device.type != "cuda":
                raise ValueError("frame inputs must be contiguous device tensors (f32, u8, f64, f64)")
        _, H, W = depth.shape
        if n and self.world == 1:  # one process: the back-projection result is the graph input as it is
            self.ctx.backproject(None, None, None, None, params, shape=(n, H, W),
                                 device_ptrs=(depth.data_ptr(), seg.data_ptr(), intrinsics.data_ptr(),
                                              poses.data_ptr()))
            col, lab, off = self.ctx.bp_mask_index()
            self.mask_index = (col, lab, off)
            self._pts = None
            self.ctx.use_backprojection()
            return col, lab, off
        if n:
            self.ctx.backproject(None, None, None, None, params, shape=(n, H, W),
                                 device_ptrs=(depth.data_ptr(), seg.data_ptr(), intrinsics.data_ptr(),
                                              poses.data_ptr()))
            col, lab, off = self.ctx.bp_mask_index()
            local = torch.empty(max(int(off[-1]), 1), dtype=torch.int32, device=depth.device)
            self.ctx.bp_points_to_device(local.data_ptr())
            self.ctx.synchronize()
        else:  # more ranks than frames
            col, lab, off = np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros(1, np.int64)
            local = torch.zeros(1, dtype=torch.int32, device=depth.device)
        g_col, g_lab, g_off, self.pts = gather_masks(col, lab, off, local, self.lo, self.group)
        self.mask_index = (g_col, g_lab, g_off)
        torch.cuda.current_stream(self.pts.device).synchronize()  # the context stream reads them next
        self.run.set_masks(self.P, self.F, g_col, g_lab, g_off, pts_device_ptr=self.pts.data_ptr())
        return g_col, g_lab, g_off

    def step(self, mask_visible_threshold, undersegment_filter_threshold, view_consensus_threshold,
             contained_threshold):
        runner = self.graph if self.graph is not None else self.run
        runner.step(mask_visible_threshold, undersegment_filter_threshold, view_consensus_threshold,
                    contained_threshold)
