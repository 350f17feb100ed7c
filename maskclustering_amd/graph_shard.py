"""Row-block sharding of the graph stages over processes (BASELINE north_star).

One process per GPU, every rank holding the same scene (the global masks, after the frame-sharded
back-projection's all-gather in ``frame_shard.py``).  The work that grows with the scene is split:

* S3 ``process_masks`` (graph/construction.py:137-170): each rank evaluates a contiguous block of
  mask rows (blocks of about equal point counts); the rows are all-gathered;
* S4 ``get_observer_num_thresholds`` (:80-96): each rank histograms every world-th tile of the
  M x M observer counts; the histograms are summed with one int64 all-reduce (the sum of the
  histograms of disjoint pair sets is the histogram of the union, unlike a histogram of sums);
* S6 iteration 0 (graph/iterative_clustering.py:20-29, the N0 x N0 pair evaluation): each rank
  evaluates the rows a = rank (mod world) into its own union-find forest; the forests (one root
  per node) are all-gathered and united on every rank, so the components are identical
  everywhere.  The later iterations (N ~ N0 / 8 and shrinking) run replicated.

No N x N count matrix is ever exchanged: at C3 the dense all-reduce would be ~51 GB, the
exchanges here are ~13 MB (S3 rows), 12 KB (histogram) and 4·N0 bytes per rank (forest).

The collectives are torch.distributed's (RCCL over xGMI under "nccl"; gloo for the tests, where
blocks go through host memory).  The library (``mc_shard_*`` in include/mcgraph.h) only packs and
unpacks the blocks, on its stream; a context whose stream is not torch's current stream is
synchronised around each exchange.  With ``native_comm=True`` the library owns an RCCL
communicator instead (``mc_ctx_comm_init``; the unique id is broadcast over ``group``) and runs
the same exchanges itself inside mc_graph_build / mc_cluster_run, stream-ordered, with nothing
left pending for the host.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

S3, HIST, FOREST = 1, 2, 3


class ShardedGraph:
    """Drives one rank's context through the sharded S2-S6 (``run``: a pipeline.GraphRun, or any
    object with a ``ctx`` exposing the mc_shard_* methods; ``group``: the process group)."""

    def __init__(self, run, group=None, native_comm=False):
        self.run = run
        self.ctx = run.ctx
        self.group = group
        on = dist.is_initialized()
        self.rank = dist.get_rank(group) if on else 0
        self.world = dist.get_world_size(group) if on else 1
        self.dev = self.ctx.torch_device
        self.comm_dev = self.dev if on and dist.get_backend(group) == "nccl" else torch.device("cpu")
        self.native = bool(native_comm)
        if self.native:
            self._comm_init()
        else:
            self.ctx.shard_set(self.rank, self.world)
        self.bytes_moved = 0

    def _comm_init(self):
        from ._native import MC_COMM_ID_BYTES, comm_unique_id
        uid = torch.zeros(MC_COMM_ID_BYTES, dtype=torch.uint8)
        if self.rank == 0:
            uid = torch.tensor(list(comm_unique_id()), dtype=torch.uint8)
        if self.world > 1:
            t = uid.to(self.comm_dev)
            dist.broadcast(t, 0, group=self.group)
            uid = t.cpu()
        self.ctx.comm_init(bytes(uid.tolist()), self.rank, self.world)

    def _same_stream(self):
        if self.dev.type != "cuda":
            return True
        return int(self.ctx.stream() or 0) == int(torch.cuda.current_stream(self.dev).cuda_stream)

    def _sync_in(self):   # the context's writes are visible to torch's stream
        if not self._same_stream():
            self.ctx.synchronize()

    def _sync_out(self):  # torch's writes are visible to the context's stream
        if not self._same_stream():
            torch.cuda.current_stream(self.dev).synchronize()

    def drain(self):
        """Run every exchange the context is waiting for (S3 -> HIST after a build, FOREST after
        a cluster run)."""
        while True:
            ph = self.ctx.shard_pending()
            if ph == 0:
                return
            if self.world == 1:
                raise RuntimeError("exchange pending in a single-process run")
            self._exchange(ph)

    def _exchange(self, ph):
        n = self.ctx.shard_export_size(ph)
        if ph == HIST:
            buf = torch.empty(n // 8, dtype=torch.int64, device=self.dev)
            self._sync_out()
            self.ctx.shard_export(ph, buf)
            self._sync_in()
            t = buf.to(self.comm_dev)
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
            t = t.to(self.dev)
            self._sync_out()
            self.ctx.shard_import(ph, t, 0)
            self.bytes_moved += n
        else:
            if ph == S3:  # variable size: the largest block sets the stride (one max-reduce, one read)
                sz = torch.tensor([n], dtype=torch.int64, device=self.comm_dev)
                dist.all_reduce(sz, op=dist.ReduceOp.MAX, group=self.group)
                n_max = int(sz.item())
            else:         # FOREST: 4·(N0 + 2) bytes on every rank
                n_max = n
            words = max((n_max + 3) // 4, 1)
            buf = torch.zeros(words, dtype=torch.int32, device=self.dev)
            self._sync_out()
            self.ctx.shard_export(ph, buf)
            self._sync_in()
            src = buf.to(self.comm_dev)
            blocks = torch.empty(self.world * words, dtype=torch.int32, device=self.comm_dev)
            dist.all_gather_into_tensor(blocks, src, group=self.group)
            blocks = blocks.to(self.dev)
            self._sync_out()
            self.ctx.shard_import(ph, blocks, 4 * words)
            self.bytes_moved += 4 * words * self.world
        if not self._same_stream():
            self.ctx.synchronize()  # the imported blocks are read before torch may reuse them

    # ---- edges of the clustering run (for the reference's container orders) -----------------
    def set_edge_capture(self, capacity):
        self.ctx.set_edge_capture(capacity)
        self._edge_cap = int(capacity)

    def _local_edges(self):
        """this rank's capture, or None when it overflowed the capacity (MC_ERR_UNSUPPORTED)"""
        from ._native import McError, MC_ERR_UNSUPPORTED
        try:
            return self.ctx.edges()
        except McError as e:
            if e.code != MC_ERR_UNSUPPORTED:
                raise
            return None

    def _any_rank(self, flag):
        """max of an int over the ranks (every rank must call it)"""
        t = torch.tensor([int(flag)], dtype=torch.int64, device=self.comm_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return int(t.item())

    def cluster_with_edges(self, connect_threshold, thresholds=None, capacity=1 << 20):
        """cluster() with every iteration's edges captured: a rank whose capture overflowed makes every
        rank grow the capacity (to the edges found, all-reduced) and re-run S6 on the same level-0
        nodes, so no rank enters edges()' collectives with a failed capture.  Returns edges()."""
        cap = int(capacity)
        while True:
            self.set_edge_capture(cap)
            self.cluster(connect_threshold, thresholds)
            local = self._local_edges()
            need = self._any_rank(0 if local is not None else 2 * cap)
            if need == 0:
                return self.edges(_local=local)
            cap = need

    def edges(self, _local=None):
        """Every iteration's edges as (t, a, b) int64 arrays sorted by (t, a, b), the same on every
        rank: iteration 0's come from the ranks' pair rows (each rank captured its own rows' edges,
        all-gathered here), the later iterations ran replicated (this rank's capture).  A rank whose
        capture overflowed its capacity makes every rank raise (checked before any exchange, so no
        rank waits in a collective the failed one never joins); cluster_with_edges grows instead."""
        import numpy as np
        from ._native import McError, MC_ERR_UNSUPPORTED
        local = _local if _local is not None else self._local_edges()
        if self.world == 1:
            if local is None:
                raise McError(MC_ERR_UNSUPPORTED, "edge capture overflowed its capacity")
            return local
        if self._any_rank(local is None):
            raise McError(MC_ERR_UNSUPPORTED, "edge capture overflowed its capacity on a rank")
        tt, aa, bb = local
        z = tt == 0
        key = ((aa[z] << 24) | bb[z]).astype(np.int64)
        n = torch.tensor([len(key)], dtype=torch.int64, device=self.comm_dev)
        dist.all_reduce(n, op=dist.ReduceOp.MAX, group=self.group)
        w = max(int(n.item()), 1)
        buf = torch.full((w,), -1, dtype=torch.int64)
        buf[:len(key)] = torch.from_numpy(key)
        allk = torch.empty(self.world * w, dtype=torch.int64, device=self.comm_dev)
        dist.all_gather_into_tensor(allk, buf.to(self.comm_dev), group=self.group)
        allk = allk.cpu().numpy()
        allk = np.unique(allk[allk >= 0])
        self.bytes_moved += 8 * w * self.world
        t0 = np.zeros(len(allk), np.int64)
        return (np.concatenate([t0, tt[~z]]), np.concatenate([allk >> 24, aa[~z]]),
                np.concatenate([allk & 0xFFFFFF, bb[~z]]))

    # ---- the reference-shaped steps ----------------------------------------------------------
    def build(self, mask_visible_threshold, contained_threshold, undersegment_filter_threshold):
        self.ctx.build(mask_visible_threshold, contained_threshold, undersegment_filter_threshold)
        self.drain()

    def cluster(self, connect_threshold, thresholds=None):
        self.ctx.cluster(thresholds, connect_threshold)
        self.drain()

    def step(self, mask_visible_threshold, undersegment_filter_threshold, view_consensus_threshold,
             contained_threshold):
        """S2-S6 (+ final point sets), the same result on every rank as GraphRun.step."""
        self.build(mask_visible_threshold, contained_threshold, undersegment_filter_threshold)
        self.cluster(view_consensus_threshold)
