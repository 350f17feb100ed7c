"""Frame-sharded scenes over ranks (BASELINE north_star).

One process per GPU.  Rank r owns a contiguous frame slice (``frame_slice``: equal frame
counts, or ``balanced_frame_slices`` over per-frame S1 cost estimates, ``frame_costs``, so that
the ranks get equal work rather than equal frames) and runs S1 (``utils/mask_backprojection.py:70-151``, per frame and independent across
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

import time

import numpy as np
import torch
import torch.distributed as dist


def frame_slice(num_frames: int, world: int, rank: int, costs=None) -> tuple[int, int]:
    """[lo, hi) of the frames rank owns: contiguous and ascending over the ranks.  Without costs
    the sizes differ by at most one frame; with a per-frame cost vector (``frame_costs``) the
    cuts fall where the cost prefix sum crosses r / world of the total, so every rank gets about
    the same S1 work (frames differ: mask pixels and voxels vary with what a frame sees)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    if costs is not None:
        return balanced_frame_slices(costs, world)[rank]
    base, extra = divmod(int(num_frames), world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def balanced_frame_slices(costs, world: int) -> list[tuple[int, int]]:
    """Contiguous frame slices of about equal total cost: cut r sits at the first frame whose
    cost prefix sum (exclusive) reaches r / world of the total, nudged to the closer side of that
    frame.  Costs are non-negative; an all-zero vector falls back to equal frame counts."""
    c = np.asarray(costs, np.float64).reshape(-1)
    F = len(c)
    if world < 1:
        raise ValueError(f"bad world size {world}")
    if not np.all(np.isfinite(c)) or np.any(c < 0):
        raise ValueError("frame costs must be finite and non-negative")
    tot = float(c.sum())
    if tot <= 0.0:
        return [frame_slice(F, world, r) for r in range(world)]
    incl = np.cumsum(c)
    excl = incl - c
    cuts = [0]
    for r in range(1, world):
        target = tot * r / world
        i = int(np.searchsorted(incl, target, side="left"))  # frame i straddles the target
        if i >= F:
            cut = F
        else:  # cut before frame i or after it, whichever lands closer to the target
            cut = i if target - excl[i] <= incl[i] - target else i + 1
        cuts.append(min(max(cut, cuts[-1]), F))
    cuts.append(F)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def frame_costs(depth, seg, intrinsics, voxel_size: float = 0.01, depth_trunc: float = 20.0,
                pixel_weight: float = 1.0, voxel_weight: float = 37.0, frame_weight: float = 2.4e5):
    """Per-frame S1 cost estimate (float64 [F], on the frames' device) for ``balanced_frame_slices``.

    S1's groups scale with three things per frame: the frame's pixels (the pixel
    count, a constant per frame), the mask pixels (voxelisation) and the voxels (denoise and
    ball query, the bulk).  Mask pixels are those with a mask id and a valid depth
    (``get_depth_mask``, utils/mask_backprojection.py:42-45); the voxels are estimated from
    the pixels' footprints: a pixel at depth d covers (d / fx)(d / fy) m², i.e. that over
    voxel_size² voxels, at most one.  The default weights are the measured C3 per-unit costs
    relative to a mask pixel (profiles/r02/v54_bench_e2e_c3.json stage times over the scene's
    pixel, mask-pixel and voxel totals)."""
    import torch
    d = depth.to(torch.float32)
    m = (seg != 0) & (d > 0) & (d <= depth_trunc)
    K = torch.as_tensor(intrinsics, dtype=torch.float64, device=d.device).reshape(-1, 4)
    fxy = (K[:, 0] * K[:, 1]).to(torch.float32).view(-1, 1, 1)
    foot = torch.clamp(d * d / (fxy * float(voxel_size) ** 2), max=1.0)
    px = m.sum(dim=(1, 2)).to(torch.float64)
    vox = torch.where(m, foot, torch.zeros_like(foot)).sum(dim=(1, 2)).to(torch.float64)
    return frame_weight + pixel_weight * px + voxel_weight * vox


def gather_frame_costs(local_costs, num_frames: int, group=None) -> np.ndarray:
    """All-gather the per-frame costs each rank computed over its equal-count slice
    (``frame_slice`` without costs) into the scene's cost vector (host float64 [F])."""
    import torch
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    lo, hi = frame_slice(num_frames, world, rank)
    t = torch.as_tensor(local_costs, dtype=torch.float64).reshape(-1)
    if len(t) != hi - lo:
        raise ValueError(f"rank {rank} holds {len(t)} frame costs, its slice is [{lo}, {hi})")
    if world == 1:
        return t.cpu().numpy()
    dev = _comm_device(group, t.device)
    width = -(-int(num_frames) // world)  # slices differ by at most one frame
    buf = torch.zeros(width, dtype=torch.float64, device=dev)
    buf[:len(t)] = t.to(dev)
    out = torch.empty(world * width, dtype=torch.float64, device=dev)
    dist.all_gather_into_tensor(out, buf, group=group)
    out = out.cpu().numpy().reshape(world, width)
    return np.concatenate([out[r, :frame_slice(num_frames, world, r)[1] - frame_slice(num_frames, world, r)[0]]
                           for r in range(world)])


def _comm_device(group, like: torch.device) -> torch.device:
    """Tensors for the collective: device tensors under RCCL ("nccl": ``like`` when it is a GPU,
    else the current GPU, so host inputs work too), host tensors under gloo."""
    if dist.get_backend(group) != "nccl":
        return torch.device("cpu")
    return like if like.type == "cuda" else torch.device("cuda", torch.cuda.current_device())


# backends whose torch.distributed gather the scene-owner path uses (RCCL "nccl" implements it over
# point-to-point sends, gloo natively); any other backend all-gathers and keeps the owner's share.
# Decided from the group's backend, which every rank reads the same, so all ranks take one branch.
_GATHER_BACKENDS = ("nccl", "gloo")


def _gather_supported(group=None) -> bool:
    return str(dist.get_backend(group)) in _GATHER_BACKENDS


def gather_masks(mask_col, mask_label, mask_off, mask_pts: torch.Tensor, frame_lo: int, group=None,
                 max_masks: int | None = None, points_ready=None, dst: int | None = None):
    """All-gather per-rank mask CSRs into the global one (dst: group rank that alone receives
    the point ids; the others get None for them).

    mask_col / mask_label / mask_off: this rank's masks (numpy; mask_col relative to
    frame_lo); mask_pts: int32 tensor of their point ids (any device).  max_masks bounds any
    rank's mask count (the default: 255 masks per frame of the largest slice, as segmentation
    ids are uint8), which fixes the size of the first collective; None (masks from any source)
    takes one max-reduce of the counts first.
    Returns (mask_col, mask_label, mask_off int64) as numpy and the global point ids as an
    int32 tensor on mask_pts' device.

    Two collectives, one host read: (1) one packed int32 block per rank, [M, nnz, col[M],
    label[M], len[M]] at a fixed stride, whose copy to the host the caller needs anyway (the
    graph input's mask index is host metadata); (2) the point ids at the largest rank's nnz,
    gathered on the device into one tensor and compacted there (with dst: gathered to that rank
    only, 1/world of the all-gather's traffic; the scene-owner pipeline).  points_ready (optional) is
    called between the two: the metadata exchange runs while mask_pts is still being written
    (e.g. by a copy on another stream that points_ready then orders torch's stream behind).
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
        if points_ready is not None:
            points_ready()
        return col, lab, off.copy(), mask_pts[:nnz].clone()
    if nnz >= 2 ** 31:
        raise ValueError("a rank's mask point ids exceed the int32 block")
    dev = _comm_device(group, out_dev)
    if max_masks is None:  # no bound known (masks from any source): one max-reduce of the counts
        mm = torch.tensor([M], dtype=torch.int64, device=dev)
        dist.all_reduce(mm, op=dist.ReduceOp.MAX, group=group)
        max_masks = int(mm.item())
    if M > max_masks:
        raise ValueError(f"{M} masks exceed the block bound {max_masks}")
    stride = 2 + 3 * int(max_masks)
    blk = np.zeros(stride, np.int32)
    blk[0], blk[1] = M, nnz
    blk[2:2 + M], blk[2 + M:2 + 2 * M], blk[2 + 2 * M:2 + 3 * M] = col, lab, np.diff(off)
    meta = torch.empty(world * stride, dtype=torch.int32, device=dev)
    dist.all_gather_into_tensor(meta, torch.from_numpy(blk).to(dev), group=group)
    meta = meta.cpu().numpy().reshape(world, stride)
    Ms, Ns = meta[:, 0].astype(np.int64), meta[:, 1].astype(np.int64)
    g_col = np.concatenate([meta[r, 2:2 + Ms[r]] for r in range(world)]).astype(np.int32)
    g_lab = np.concatenate([meta[r, 2 + Ms[r]:2 + 2 * Ms[r]] for r in range(world)]).astype(np.int32)
    g_len = np.concatenate([meta[r, 2 + 2 * Ms[r]:2 + 3 * Ms[r]] for r in range(world)]).astype(np.int64)
    g_off = np.zeros(len(g_len) + 1, np.int64)
    np.cumsum(g_len, out=g_off[1:])
    nmax = max(1, int(Ns.max()))
    if points_ready is not None:
        points_ready()
    buf = torch.zeros(nmax, dtype=torch.int32, device=dev)
    buf[:nnz] = mask_pts[:nnz].to(dev)
    if dst is not None and _gather_supported(group):
        me = dist.get_rank(group)
        gdst = dst if group is None else dist.get_global_rank(group, dst)
        parts = [torch.empty(nmax, dtype=torch.int32, device=dev) for _ in range(world)] if me == dst else None
        dist.gather(buf, parts, dst=gdst, group=group)
        if me != dst:
            return g_col, g_lab, g_off, None
        return g_col, g_lab, g_off, torch.cat([parts[r][:int(Ns[r])] for r in range(world)]).to(out_dev)
    allp = torch.empty(world * nmax, dtype=torch.int32, device=dev)
    dist.all_gather_into_tensor(allp, buf, group=group)
    allp = allp.view(world, nmax).to(out_dev)
    if dst is not None and dist.get_rank(group) != dst:
        return g_col, g_lab, g_off, None
    g_pts = torch.cat([allp[r, :int(Ns[r])] for r in range(world)])
    return g_col, g_lab, g_off, g_pts


def _check_same_on_all_ranks(costs: np.ndarray, group=None):
    """Raise on every rank if the ranks hold different cost vectors (their slices would overlap or
    leave frames out, and gather_masks would concatenate them without an error): a min and a max
    all-reduce of an order-sensitive checksum of the float64 bits."""
    bits = costs.view(np.uint64)
    w = np.arange(1, len(bits) + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
    h = int(np.bitwise_xor.reduce(bits * w) if len(bits) else 0) & ((1 << 62) - 1)
    dev = _comm_device(group, torch.device("cpu"))
    lo = torch.tensor([h], dtype=torch.int64, device=dev)
    hi = lo.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=group)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=group)
    if int(lo.item()) != int(hi.item()):
        raise ValueError("the ranks hold different frame cost vectors: their frame slices would disagree")


def rccl_comm_ranks(group=None):
    """The rank count RCCL's own communicator of the group reports (ncclCommCount on the communicator
    torch's "nccl" backend made, from torch's librccl), or None: another backend, or no communicator
    yet (it is made by the first collective on the device)."""
    import ctypes
    import os
    if not dist.is_initialized() or dist.get_backend(group) != "nccl":
        return None
    pg = group if group is not None else dist.distributed_c10d._get_default_group()
    try:
        ptr = int(pg._get_backend(torch.device("cuda", torch.cuda.current_device()))._comm_ptr())
    except (RuntimeError, AttributeError):
        return None
    if not ptr:
        return None
    lib = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so"))
    cnt = ctypes.c_int(0)
    return int(cnt.value) if lib.ncclCommCount(ctypes.c_void_p(ptr), ctypes.byref(cnt)) == 0 else None


def _stream_wait(stream: int, cur, device):
    """Make HIP stream `stream` (a library context's; 0 = the null stream) wait on torch stream
    `cur` on the device: an event, no host wait (the null stream waits on the host)."""
    if stream == int(cur.cuda_stream):
        return
    if stream == 0:
        cur.synchronize()
        return
    torch.cuda.ExternalStream(stream, device=device).wait_stream(cur)


class FrameShardedScene:
    """S1 on this rank's frames, all-gather, then the replicated graph path.

    ``run`` is this rank's :class:`maskclustering_amd.pipeline.GraphRun` (its context holds
    the scene points: ``ctx.set_points``).  Inputs of :meth:`backproject` are this rank's
    frame slice, resident on its GPU.
    """

    def __init__(self, run, num_points: int, num_frames: int, group=None, shard_graph: bool = True,
                 costs=None, native_comm: bool = False):
        from .graph_shard import ShardedGraph
        self.run = run
        self.ctx = run.ctx
        self.P, self.F = int(num_points), int(num_frames)
        self.group = group
        on = dist.is_initialized()
        self.rank = dist.get_rank(group) if on else 0
        self.world = dist.get_world_size(group) if on else 1
        # costs (per-frame, e.g. gather_frame_costs(frame_costs(...))): cost-balanced slices; every
        # rank must cut the same slices, so the cost vectors are compared across the ranks first
        if costs is not None:
            costs = np.asarray(costs, np.float64).reshape(-1)
            if len(costs) != self.F:
                raise ValueError(f"{len(costs)} frame costs for {self.F} frames")
            if self.world > 1:
                _check_same_on_all_ranks(costs, group)
        self.slices = (balanced_frame_slices(costs, self.world) if costs is not None
                       else [frame_slice(self.F, self.world, r) for r in range(self.world)])
        self.lo, self.hi = self.slices[self.rank]
        # the mask block bound of gather_masks for S1 output: 255 ids per frame of the largest slice
        self.max_masks = 255 * max(1, max(hi - lo for lo, hi in self.slices))
        self._pts = None  # global point ids (kept alive until the graph input copy is done)
        # the graph stages row-block sharded over the same ranks (shard_graph=False: replicated)
        # (native_comm: the graph stages' exchanges run inside the library over its own RCCL
        # communicator, mc_ctx_comm_init, instead of torch.distributed collectives between calls)
        self.graph = ShardedGraph(run, group, native_comm=native_comm) if shard_graph else None

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
                    poses: torch.Tensor, params=None, s1_ctx=None):
        """depth f32 [n,H,W], seg u8 [n,H,W], intrinsics f64 [n,4], poses f64 [n,16] on this
        rank's GPU, n = hi - lo.  Leaves the global masks as the graph input.  s1_ctx (optional): the
        context S1 runs on (its scene points set), instead of the graph context."""
        n = self.hi - self.lo
        if depth.shape[0] != n or seg.shape != depth.shape or intrinsics.shape[0] != n or poses.shape[0] != n:
            raise ValueError(f"rank {self.rank} owns {n} frames [{self.lo}, {self.hi})")
        for t, dt in ((depth, torch.float32), (seg, torch.uint8), (intrinsics, torch.float64),
                      (poses, torch.float64)):
            if t.dtype != dt or not t.is_contiguous() or t.device.type != "cuda":
                raise ValueError("frame inputs must be contiguous device tensors (f32, u8, f64, f64)")
        _, H, W = depth.shape
        c1 = self.ctx if s1_ctx is None else s1_ctx
        if n and self.world == 1 and c1 is self.ctx:  # one process: the back-projection result is the graph input
            self.ctx.backproject(None, None, None, None, params, shape=(n, H, W),
                                 device_ptrs=(depth.data_ptr(), seg.data_ptr(), intrinsics.data_ptr(),
                                              poses.data_ptr()))
            col, lab, off = self.ctx.bp_mask_index()
            self.mask_index = (col, lab, off)
            self._pts = None
            self.ctx.use_backprojection()
            return col, lab, off
        if n:
            c1.backproject(None, None, None, None, params, shape=(n, H, W),
                           device_ptrs=(depth.data_ptr(), seg.data_ptr(), intrinsics.data_ptr(), poses.data_ptr()))
            col, lab, off = c1.bp_mask_index()
            local = torch.empty(max(int(off[-1]), 1), dtype=torch.int32, device=depth.device)
            # the copy of the point ids runs on the S1 context's stream while the metadata block is
            # exchanged; torch's stream (the collectives') is ordered behind it without a host wait
            # (and the copy behind torch's stream: `local` may reuse a block torch's stream still reads)
            _stream_wait(int(c1.stream() or 0), torch.cuda.current_stream(depth.device), depth.device)
            c1.bp_points_to_device(local.data_ptr())
            ready = lambda: self._order_streams(torch_after_ctx=True, device=depth.device, ctx=c1)  # noqa: E731
        else:  # more ranks than frames
            col, lab, off = np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros(1, np.int64)
            local = torch.zeros(1, dtype=torch.int32, device=depth.device)
            ready = None
        g_col, g_lab, g_off, self.pts = gather_masks(col, lab, off, local, self.lo, self.group, self.max_masks,
                                                     points_ready=ready)
        self.mask_index = (g_col, g_lab, g_off)
        # the context's stream reads the gathered ids next: ordered behind torch's stream on the device
        self._order_streams(torch_after_ctx=False, device=self.pts.device)
        self.run.set_masks(self.P, self.F, g_col, g_lab, g_off, pts_device_ptr=self.pts.data_ptr())
        return g_col, g_lab, g_off

    def _order_streams(self, torch_after_ctx: bool, device, ctx=None):
        """Device-side ordering between a context's stream (default: the graph context's) and
        torch's current stream (an event recorded on one, waited on by the other); nothing when they
        are the same stream."""
        c = self.ctx if ctx is None else ctx
        cur = torch.cuda.current_stream(device)
        s = int(c.stream() or 0)
        if s == int(cur.cuda_stream):
            return
        if s == 0:  # the context runs on the null stream: a host-side join is the safe order
            (c.synchronize if torch_after_ctx else cur.synchronize)()
            return
        ext = torch.cuda.ExternalStream(s, device=device)
        (cur.wait_stream(ext) if torch_after_ctx else ext.wait_stream(cur))

    def step(self, mask_visible_threshold, undersegment_filter_threshold, view_consensus_threshold,
             contained_threshold):
        runner = self.graph if self.graph is not None else self.run
        runner.step(mask_visible_threshold, undersegment_filter_threshold, view_consensus_threshold,
                    contained_threshold)


class ScenePipeline:
    """A stream of scenes through one :class:`FrameShardedScene`, S1 of scene k + 1 overlapping the
    graph stages of scene k.

    S1 (this rank's frame slice) runs on its own context ``s1_ctx`` and stream, in a producer thread
    (the library's calls release the GIL); the calling thread takes each scene's masks, gathers
    them over the ranks (the only collectives, all issued by this thread, in the same order on every
    rank), hands them to the graph context and runs S2-S6 there.  Per scene the work is exactly the
    sequential path's (``FrameShardedScene.backproject`` + ``step``, the same results); only the
    order in time changes, so that the graph stages, which run serially on every rank after the
    gather and do not shrink with the rank count, hide under the next scene's S1.
    The producer runs at most two scenes ahead (a bounded queue of mask sets).

    ``scene_owner=True`` (several ranks): every rank still back-projects its frame slice of every
    scene, but scene k's masks are gathered to one rank only, its owner ``(first_owner + k) mod
    world``, which alone runs S2-S6 for it, unsharded, on its graph context.  The graph stages then
    cost each rank 1/world of their time per scene instead of all of it (sharding them row-block wise
    leaves S2, S6 levels >= 1 and the object extraction replicated), and the point ids
    cross the links once instead of world - 1 times.  Scenes are independent (the reference itself
    runs one scene per process, ``run.py:33-50``), so each scene's result is the single-process one,
    held by its owner (``owned``: the scene numbers this rank ran S2-S6 for).
    """

    def __init__(self, sh: FrameShardedScene, s1_ctx, depth: torch.Tensor, seg: torch.Tensor,
                 intrinsics: torch.Tensor, poses: torch.Tensor, params=None, scene_owner: bool = False,
                 scene_points: torch.Tensor | None = None):
        n = sh.hi - sh.lo
        if depth.shape[0] != n:
            raise ValueError(f"rank {sh.rank} owns {n} frames [{sh.lo}, {sh.hi})")
        self.sh = sh
        # one or more S1 contexts: with P of them, P producer threads take scenes k = i mod P each on
        # its own context and stream, so that one scene's kernel tails (a persistent ticket kernel's
        # last slots, a batch's host sync) are filled by the next scene's kernels; scenes are still
        # handed over in order
        self.s1s = list(s1_ctx) if isinstance(s1_ctx, (list, tuple)) else [s1_ctx]
        self.s1 = self.s1s[0]
        self.frames = (depth, seg, intrinsics, poses)
        self.params = params
        # scene_points (float32 [P,3] on the device, optional): handed to the S1 context before every
        # scene's back-projection, as each new scene's points are (mc_scene_set_points), so each scene
        # rebuilds its ball-query grid inside its own S1 (graph/construction.py:37, per scene)
        self.scene_points = scene_points
        self.scene_owner = bool(scene_owner) and sh.world > 1
        self.owned: list[int] = []
        self.gather_s = 0.0   # host wall time in gather_masks (both collectives) over the scenes run
        self.gathers = 0

    def warm(self):
        """One S1 call on every context but the first (a context's first call sizes its batches for
        the worst case and allocates; run(1), the bench's warmup step, only reaches the first)."""
        for c in self.s1s[1:]:
            self._s1_scene(c)

    def _s1_scene(self, s1=None):
        """S1 of this rank's slice on an S1 context: (col, lab, off, point ids on the device)."""
        s1 = self.s1 if s1 is None else s1
        depth, seg, K, T = self.frames
        n, H, W = depth.shape
        if n == 0:
            return (np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros(1, np.int64),
                    torch.zeros(1, dtype=torch.int32, device=depth.device))
        if self.scene_points is not None:
            s1.set_points(device_ptr=self.scene_points.data_ptr(), num_points=len(self.scene_points))
        s1.backproject(None, None, None, None, self.params, shape=(n, H, W),
                       device_ptrs=(depth.data_ptr(), seg.data_ptr(), K.data_ptr(), T.data_ptr()))
        col, lab, off = s1.bp_mask_index()
        # pts comes from torch's caching allocator on torch's current stream, and the block may be one
        # the consumer freed while its reads (the gather, a cat) are still queued there: the S1
        # stream writes it only after torch's stream has drained up to this point
        pts = torch.empty(max(int(off[-1]), 1), dtype=torch.int32, device=depth.device)
        if depth.device.type == "cuda":
            _stream_wait(int(s1.stream() or 0), torch.cuda.current_stream(depth.device), depth.device)
        s1.bp_points_to_device(pts.data_ptr())
        s1.synchronize()  # the ids are complete before another stream reads them
        return col, lab, off, pts

    def run(self, num_scenes: int, on_scene=None, first_owner: int = 0, **step_kwargs):
        """num_scenes scenes (each S1 -> gather -> S2-S6); on_scene(k) after scene k's graph stages
        were issued (with scene_owner: on its owner only).  Returns when the last scene's graph
        stages have been issued on the graph context's stream (synchronize it to wait for them)."""
        import queue
        import threading
        NP = len(self.s1s)
        qs = [queue.Queue(maxsize=1) for _ in range(NP)]
        stop = threading.Event()

        def produce(i):
            q = qs[i]
            try:
                for _ in range(i, num_scenes, NP):
                    item = self._s1_scene(self.s1s[i])
                    while not stop.is_set():
                        try:
                            q.put(item, timeout=0.5)
                            break
                        except queue.Full:
                            continue
                    if stop.is_set():
                        return
            except BaseException as e:  # handed to the consumer, which raises it (dropped once it stopped)
                while not stop.is_set():
                    try:
                        q.put(e, timeout=0.5)
                        break
                    except queue.Full:
                        continue

        ths = [threading.Thread(target=produce, args=(i,), name=f"s1-producer-{i}", daemon=True) for i in range(NP)]
        for th in ths:
            th.start()
        sh = self.sh
        try:
            for k in range(num_scenes):
                item = qs[k % NP].get()
                if isinstance(item, BaseException):
                    raise item
                col, lab, off, pts = item
                owner = (first_owner + k) % sh.world
                if sh.world == 1:
                    g_col, g_lab, g_off, g_pts = col, lab, off, pts
                elif self.scene_owner:
                    tg = time.perf_counter()
                    g_col, g_lab, g_off, g_pts = gather_masks(col, lab, off, pts, sh.lo, sh.group, sh.max_masks,
                                                              dst=owner)
                    self.gather_s += time.perf_counter() - tg
                    self.gathers += 1
                    if sh.rank != owner:
                        continue
                else:
                    tg = time.perf_counter()
                    g_col, g_lab, g_off, g_pts = gather_masks(col, lab, off, pts, sh.lo, sh.group, sh.max_masks)
                    self.gather_s += time.perf_counter() - tg
                    self.gathers += 1
                sh.mask_index = (g_col, g_lab, g_off)
                sh.pts = g_pts
                # the graph context's stream reads the gathered ids (written on torch's stream) next
                if g_pts.device.type == "cuda":
                    sh._order_streams(torch_after_ctx=False, device=g_pts.device)
                # set_masks copies the ids into the graph context and synchronises its stream before
                # it returns (mc_scene_set_masks validates them on the host), so the producer's
                # tensors, allocated on its thread's stream, are free to be reused afterwards
                if g_pts.device.type == "cuda":
                    sh.run.set_masks(sh.P, sh.F, g_col, g_lab, g_off, pts_device_ptr=g_pts.data_ptr())
                else:
                    sh.run.set_masks(sh.P, sh.F, g_col, g_lab, g_off, g_pts.numpy())
                if self.scene_owner:  # the whole scene on this rank: the unsharded graph stages
                    sh.run.step(step_kwargs["mask_visible_threshold"], step_kwargs["undersegment_filter_threshold"],
                                step_kwargs["view_consensus_threshold"], step_kwargs["contained_threshold"])
                    self.owned.append(k)
                else:
                    sh.step(**step_kwargs)
                if on_scene is not None:
                    on_scene(k)
        finally:
            stop.set()
            for th in ths:
                th.join()
