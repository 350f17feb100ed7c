"""A CPU stand-in for the sharded context API of libmcgraph (mc_shard_*, include/mcgraph.h), computed
with the sparse oracle (oracle/graph_sparse.c).  TEST INFRASTRUCTURE: it lets the product's
exchange driver (maskclustering_amd.graph_shard.ShardedGraph) and its collectives run over gloo on
the CPU, so the row-block decomposition (S3 row blocks, S4 histogram shares summed, S6 level-0
forests united) is checked against the single-process result without a GPU.  Block layouts follow
mc_shard_kernels.inl."""
from __future__ import annotations

import numpy as np
import torch

from oracle import oracle as orc

S3, HIST, FOREST = 1, 2, 3


class _DSU:
    """union-find with the smaller index as root (the k6 kernels' min-root hooking)"""

    def __init__(self, n):
        self.p = np.arange(n, dtype=np.int64)

    def find(self, x):
        p = self.p
        r = x
        while p[r] != r:
            r = p[r]
        while p[x] != r:
            p[x], x = r, p[x]
        return r

    def unite(self, a, b):
        a, b = self.find(a), self.find(b)
        if a != b:
            lo, hi = (a, b) if a < b else (b, a)
            self.p[hi] = lo


class OracleShardCtx:
    torch_device = torch.device("cpu")

    def __init__(self):
        self.rank, self.world, self.pending = 0, 1, 0
        self.cap = 0
        self.e0 = np.zeros(0, np.int64)
        self.later = np.zeros(0, np.uint64)

    # ---- edge capture (mc_cluster_set_edge_capture / mc_cluster_get_edges) ----
    def set_edge_capture(self, capacity):
        self.cap = int(capacity)

    def edges(self):
        """(t, a, b) sorted: iteration 0's of this rank's pair rows, the later iterations' all"""
        a0, b0 = self.e0 >> 32, self.e0 & 0xffffffff
        k = self.later
        key = np.sort(np.concatenate([(a0.astype(np.uint64) << np.uint64(24)) | b0.astype(np.uint64), k]))
        if getattr(self, "ovf", False) or len(key) > self.cap:  # an overflowed capture (mc_cluster_get_edges)
            from maskclustering_amd._native import McError, MC_ERR_UNSUPPORTED
            raise McError(MC_ERR_UNSUPPORTED, "edge capture overflowed its capacity")
        return ((key >> np.uint64(48)).astype(np.int64), ((key >> np.uint64(24)) & np.uint64(0xFFFFFF)).astype(np.int64),
                (key & np.uint64(0xFFFFFF)).astype(np.int64))

    def level0_sequences(self):
        """each level-0 node's point set as the reference made it (ascending ids), as (pt_off, pts)"""
        keep_idx = np.nonzero(self.kept)[0]
        rows = keep_idx[self.node0]
        lens = np.diff(self.off)[rows]
        po = np.zeros(len(rows) + 1, np.int64)
        np.cumsum(lens, out=po[1:])
        pts = np.concatenate([self.pts[self.off[r]:self.off[r + 1]] for r in rows]) if len(rows) else np.zeros(0, np.int32)
        return po, pts.astype(np.int32)

    # ---- context plumbing the driver reads ----
    def stream(self):
        return None

    def synchronize(self):
        pass

    def shard_set(self, rank, world):
        self.rank, self.world, self.pending = int(rank), int(world), 0

    def shard_pending(self):
        return self.pending

    def set_masks(self, num_points, num_frames, mask_col, mask_label, mask_off, mask_pts=None, pts_device_ptr=None):
        self.P, self.F = int(num_points), int(num_frames)
        self.col = np.ascontiguousarray(mask_col, np.int32)
        self.label = np.ascontiguousarray(mask_label, np.int32)
        self.off = np.ascontiguousarray(mask_off, np.int64)
        self.pts = np.ascontiguousarray(mask_pts, np.int32)

    # ---- S2 + S3 on this rank's rows ----
    def build(self, mvt, ct, ust):
        L = orc.lib()
        P, F, M_in = self.P, self.F, len(self.col)
        self.FW = max((F + 63) // 64, 1)
        kept = np.zeros(max(M_in, 1), np.uint8)
        self.bnd = np.zeros(max(P, 1), np.uint8)
        pt_off = np.zeros(P + 1, np.int64)
        pt_ent = np.zeros(max(int(self.off[-1]) if M_in else 0, 1), np.int32)
        self.M = M = L.orcs_s2(P, F, M_in, self.col, self.off, self.pts, kept, self.bnd, pt_off, pt_ent)
        self.kept = kept[:M_in]
        gidx = np.where(self.kept > 0, np.cumsum(self.kept) - 1, -1).astype(np.int32)
        # contiguous row blocks of about equal point counts (mc_api.hip build_s3_lists)
        h_off = np.zeros(M + 1, np.int64)
        np.cumsum(np.diff(self.off)[self.kept > 0], out=h_off[1:])
        tot, W = int(h_off[-1]), self.world

        def cut(k):
            if k <= 0:
                return 0
            if k >= W:
                return M
            return int(np.searchsorted(h_off, (tot * k + W - 1) // W, side="left"))

        self.r0 = min(cut(self.rank), M)
        self.r1 = max(self.r0, min(cut(self.rank + 1), M))
        own = ((gidx >= self.r0) & (gidx < self.r1)).astype(np.uint8)
        Fc = max(F, 1)
        self.Fc = Fc
        self.ct_frame = np.zeros(max(M, 1) * Fc, np.int32)
        self.ct_tgt = np.zeros(max(M, 1) * Fc, np.int32)
        self.ct_len = np.zeros(max(M, 1), np.int32)
        self.useg = np.zeros(max(M, 1), np.uint8)
        L.orcs_s3(M_in, self.col, self.label, self.off, self.pts, np.ascontiguousarray(self.kept), gidx, self.bnd,
                  pt_off, pt_ent, float(mvt), float(ct), float(ust), Fc, self.ct_frame, self.ct_tgt, self.ct_len,
                  self.useg, own.ctypes.data)
        if self.world > 1:
            self.pending = S3
        else:
            self._tail()
            self._thresholds(self.hist_part)

    def _tail(self):
        """undo + VF rows + this rank's share of the observer histogram"""
        L = orc.lib()
        M, F, Fc = self.M, self.F, self.Fc
        L.orcs_undo(M, Fc, self.ct_frame, self.ct_tgt, self.ct_len, self.useg)
        cf, tg = self.ct_frame.reshape(-1, Fc), self.ct_tgt.reshape(-1, Fc)
        lens = self.ct_len[:M]
        self.c_rows = np.repeat(np.arange(M), lens)
        cc = np.concatenate([cf[r, :lens[r]] for r in range(M)]) if M else np.zeros(0, np.int32)
        self.c_tgts = np.concatenate([tg[r, :lens[r]] for r in range(M)]) if M else np.zeros(0, np.int32)
        vfw = np.zeros((max(M, 1), self.FW), np.uint64)
        if len(cc):
            np.bitwise_or.at(vfw, (self.c_rows, cc // 64), np.left_shift(np.uint64(1), (cc % 64).astype(np.uint64)))
        self.vfw = np.ascontiguousarray(vfw[:M] if M else vfw)
        self.hist_part = np.zeros(F + 1, np.uint64)
        L.orcs_observer_hist(M, self.FW, self.vfw, self.hist_part, F, self.rank, self.world)

    def _thresholds(self, hist):
        self.hist = np.asarray(hist, np.uint64)
        self.thr, self.thr_isint = orc.thresholds_from_hist(self.hist)
        self.pending = 0

    # ---- S6 with iteration 0 on this rank's rows ----
    def cluster(self, thresholds, connect_threshold):
        L = orc.lib()
        M, FW = self.M, self.FW
        self.ct = float(connect_threshold)
        thr = self.thr if thresholds is None else np.asarray(thresholds, np.float32)
        self.thr_used = np.ascontiguousarray(thr, np.float32)
        useg = self.useg[:M]
        self.node0 = np.nonzero(useg == 0)[0].astype(np.int32)
        order = np.lexsort((self.c_tgts, self.c_rows))
        rr, tt = self.c_rows[order], self.c_tgts[order]
        c_off_all = np.zeros(M + 1, np.int64)
        np.cumsum(self.ct_len[:M], out=c_off_all[1:])
        N0 = len(self.node0)
        self.c_off0 = np.zeros(N0 + 1, np.int64)
        np.cumsum(self.ct_len[self.node0].astype(np.int64), out=self.c_off0[1:])
        self.c_idx0 = np.concatenate([tt[c_off_all[g]:c_off_all[g + 1]] for g in self.node0]).astype(np.int32) \
            if N0 and self.c_off0[-1] else np.zeros(1, np.int32)
        self.vf0 = np.ascontiguousarray(self.vfw[self.node0]) if N0 else np.zeros((1, FW), np.uint64)
        del rr
        self.dsu = _DSU(N0)
        self.edges0 = 0
        if len(self.thr_used) and N0:
            cap = 1 << 16
            while True:
                e = np.zeros(cap, np.int64)
                n = L.orcs_level_edges(N0, FW, M, self.vf0, self.c_off0, np.ascontiguousarray(self.c_idx0),
                                       float(self.thr_used[0]), self.ct, self.rank, self.world, e, cap)
                if n <= cap:
                    break
                cap = int(n)
            for x in e[:n]:
                self.dsu.unite(int(x >> 32), int(x & 0xffffffff))
            self.edges0 = int(n)
            self.e0 = e[:n].copy()
            if self.world > 1:
                self.pending = FOREST
                return
        self._finish()

    def _finish(self):
        L = orc.lib()
        M, FW, N0 = self.M, self.FW, len(self.node0)
        T = len(self.thr_used)
        if T == 0:
            self.parts, self.sizes, self.final, self.edge_n = [], np.array([N0], np.int32), np.arange(N0), []
            self.vf_fin, self.c_off_fin, self.c_idx_fin = self.vf0[:N0], self.c_off0, self.c_idx0[:self.c_off0[-1]]
            return
        roots = np.array([self.dsu.find(i) for i in range(N0)], np.int64)
        uniq = np.unique(roots)                   # ascending roots = ascending smallest members
        lab0 = np.searchsorted(uniq, roots).astype(np.int32)
        K1 = len(uniq)
        vf1 = np.zeros((max(K1, 1), FW), np.uint64)
        np.bitwise_or.at(vf1, lab0, self.vf0[:N0])
        rows = [[] for _ in range(K1)]
        for i in range(N0):
            rows[lab0[i]].append(self.c_idx0[self.c_off0[i]:self.c_off0[i + 1]])
        rows = [np.unique(np.concatenate(r)).astype(np.int32) if r else np.zeros(0, np.int32) for r in rows]
        co1 = np.zeros(K1 + 1, np.int64)
        np.cumsum([len(r) for r in rows], out=co1[1:])
        ci1 = np.concatenate(rows).astype(np.int32) if co1[-1] else np.zeros(1, np.int32)
        T1 = T - 1
        labels = np.full((max(T1, 1), max(K1, 1)), -1, np.int32)
        sizes1 = np.zeros(T1 + 1, np.int32)
        final1 = np.zeros(max(K1, 1), np.int32)
        edges1 = np.zeros(max(T1, 1), np.int64)
        vf_out = np.zeros((max(K1, 1), FW), np.uint64)
        co_out = np.zeros(max(K1, 1) + 1, np.int64)
        ci_out = np.zeros(max(int(co1[-1]), 1), np.int32)
        sink = np.zeros(max(self.cap, 1), np.uint64)
        if self.cap:
            L.orcs_set_edge_sink(sink.ctypes.data, self.cap)
        try:
            K = L.orcs_cluster(K1, FW, M, np.ascontiguousarray(vf1), co1, np.ascontiguousarray(ci1), T1,
                               np.ascontiguousarray(self.thr_used[1:]), self.ct, labels, sizes1, final1, edges1, vf_out,
                               co_out, ci_out)
            n = L.orcs_edge_sink_count() if self.cap else 0
        finally:
            L.orcs_set_edge_sink(None, 0)
        self.ovf = bool(self.cap) and n > self.cap  # (the library keeps the first cap edges and reports it)
        k = sink[:min(n, self.cap)]   # iteration t of this call is iteration t + 1 of the run
        self.later = ((((k >> np.uint64(48)) + np.uint64(1)) << np.uint64(48)) | (k & np.uint64((1 << 48) - 1))).astype(np.uint64)
        self.parts = [lab0] + [labels[t, :sizes1[t]].copy() for t in range(T1)]
        self.sizes = np.concatenate([[N0], sizes1]).astype(np.int32)
        self.final = final1[lab0]
        self.edge_n = [self.edges0] + edges1[:T1].tolist()
        self.vf_fin, self.c_off_fin, self.c_idx_fin = vf_out[:K], co_out[:K + 1], ci_out[:co_out[K]]

    # ---- exchange blocks ----
    def shard_export_size(self, phase):
        return self._block(phase).nbytes

    def shard_export(self, phase, out):
        b = self._block(phase)
        out.view(torch.uint8)[:b.nbytes] = torch.from_numpy(b.view(np.uint8))

    def _block(self, phase):
        if phase == S3:
            r0, r1 = self.r0, self.r1
            tg = self.ct_tgt.reshape(-1, self.Fc)
            ent = [tg[r, :self.ct_len[r]] for r in range(r0, r1)]
            return np.concatenate([[r0, r1], self.ct_len[r0:r1], self.useg[r0:r1].astype(np.int32)] + ent).astype(np.int32)
        if phase == HIST:
            return self.hist_part.view(np.int64).copy()
        if phase == FOREST:
            N0 = len(self.node0)
            roots = np.array([self.dsu.find(i) for i in range(N0)], np.int64)
            e = np.int64(self.edges0)
            return np.concatenate([roots, [e & 0xffffffff, e >> 32]]).astype(np.int32)
        raise ValueError(phase)

    def shard_import(self, phase, blocks, stride_bytes):
        a = blocks.numpy()
        if phase == S3:
            w = a.view(np.int32).reshape(self.world, stride_bytes // 4)
            tg = self.ct_tgt.reshape(-1, self.Fc)
            for r in range(self.world):
                if r == self.rank:
                    continue
                b = w[r]
                r0, r1 = int(b[0]), int(b[1])
                nr = r1 - r0
                lens, flg = b[2:2 + nr], b[2 + nr:2 + 2 * nr]
                o = 2 + 2 * nr
                for i in range(nr):
                    self.ct_len[r0 + i] = lens[i]
                    self.useg[r0 + i] = flg[i]
                    tg[r0 + i, :lens[i]] = b[o:o + lens[i]]
                    self.ct_frame.reshape(-1, self.Fc)[r0 + i, :lens[i]] = self.col[np.nonzero(self.kept)[0]][b[o:o + lens[i]]]
                    o += lens[i]
            self._tail()
            self.pending = HIST
        elif phase == HIST:
            self._thresholds(a.view(np.int64).view(np.uint64))
        elif phase == FOREST:
            N0 = len(self.node0)
            w = a.view(np.int32).reshape(self.world, stride_bytes // 4)
            for r in range(self.world):
                if r == self.rank:
                    continue
                for i, root in enumerate(w[r, :N0]):
                    if root != i:
                        self.dsu.unite(i, int(root))
                self.edges0 += int(np.uint32(w[r, N0])) | (int(np.uint32(w[r, N0 + 1])) << 32)
            self.pending = 0
            self._finish()
        else:
            raise ValueError(phase)

    def canonical(self):
        return orc.assemble_sparse(self.P, self.F, self.col, self.label, self.off, self.pts, self.kept, self.bnd,
                                   self.c_rows, self.c_tgts, self.useg[:self.M], self.vfw, self.hist, self.thr,
                                   self.thr_isint, self.node0, self.parts, self.sizes, self.final, self.edge_n,
                                   self.vf_fin, self.c_off_fin, self.c_idx_fin)
