"""Drop-in for the reference's ``graph/iterative_clustering.py`` (S6).

``iterative_clustering(nodes, observer_num_thresholds, connect_threshold,
debug)`` keeps the reference's signature and result (iterative_clustering.py
:36-43): the final list of merged ``Node`` objects, in ascending order of their
smallest initial node (the order of nx.connected_components, :7), with
``node_info = (iterations, k)`` and ``son_node_info`` = the node_info of the
members of the last iteration.  Every iteration runs on the device
(mc_cluster_run: pair consensus counts, the float32 edge rule, union-find,
on-device merge).  Nodes that come straight from this package's
``mask_graph_construction`` are clustered from the device graph without a
host round trip; any other node list is packed into CSR rows first.

Container orders.  The reference's ``Node.mask_list`` order and ``point_ids``
iteration order follow CPython's set tables (networkx's BFS ``seen`` set, iterative_clustering.py:7;
the chained ``set.union``, graph/node.py:31-36), and post_process numbers its DBSCAN objects by
``list(point_ids)`` (graph/node.py:45), so the exports depend on them.

* reference order (default): the device also records every edge of every iteration; the host
  restates what the reference's Python does with them natively (``mc_setorder_replay``: networkx
  3.x's ``_plain_bfs`` + CPython's set tables, include/mcgraph.h), so ``mask_list`` is the
  reference's list and ``point_ids`` a set that iterates in the reference's order
  (node.RefOrderSet); post_process then exports exactly what the reference exports
  (tests/test_gpu_api.py, golden from the reference's own S1 -> S6 -> post_process;
  tests/test_setorder_cpu.py against the interpreter).  Node lists that do not come from this
  package's ``mask_graph_construction`` (point sets of unknown history) take the same steps with
  real Python sets (``_replay``).
* canonical (``replay=False``, or MASKCLUSTERING_SET_ORDER=canonical): contents only -- a merged
  node's ``mask_list`` in ascending member order and ``point_ids`` built from the device's sorted
  ids; no edge capture, no host replay.
"""
from __future__ import annotations

import operator
import os

import numpy as np

from .. import _device, _native
from .._hostutil import no_gc
from ..pipeline import bits_to_bool, bool_to_bits
from .node import Node, level0_masks


def _fast_path(nodes):
    from . import construction
    if not nodes:
        return None
    h = getattr(nodes[0], "_graph", None)
    if h is None or h.token != construction._current["token"] or len(nodes) != h.num_nodes:
        return None
    # the same level-0 Node objects in the same order (a C-speed identity scan), none of them with a
    # replaced visible_frame / contained_mask (the setters mark the handle touched)
    if h.touched or not all(map(operator.is_, nodes, h.nodes)):
        return None
    return h


def _pack(ctx, nodes):
    F = len(nodes[0].visible_bool())
    M = nodes[0].num_masks()
    vf = np.stack([n.visible_bool() for n in nodes])
    cids = [n.contained_ids() for n in nodes]
    c_off = np.zeros(len(nodes) + 1, np.int64)
    np.cumsum([len(c) for c in cids], out=c_off[1:])
    pts = [np.sort(np.fromiter(n.point_ids, dtype=np.int64)) for n in nodes]
    p_off = np.zeros(len(nodes) + 1, np.int64)
    np.cumsum([len(p) for p in pts], out=p_off[1:])
    P = int(max((int(p[-1]) + 1 for p in pts if len(p)), default=1))
    ctx.set_nodes(F, M, P, bool_to_bits(vf), c_off, np.concatenate(cids).astype(np.int32) if cids else
                  np.zeros(0, np.int32), p_off, np.concatenate(pts).astype(np.int32) if pts else np.zeros(0, np.int32))
    return F, M


REFERENCE_SET_ORDER = os.environ.get("MASKCLUSTERING_SET_ORDER", "reference").lower() != "canonical"
REPLAY_SET_ORDER = REFERENCE_SET_ORDER  # (round-3 name)
_EDGE_CAP0 = 1 << 22


def _replay(nodes, T, sizes, edges, parts):
    """The reference's container building, level by level (see the module docstring).  Returns
    [(mask_list, point_ids, son_node_info)] of the final nodes, in component order.

    The component walk is networkx 3.x's ``_plain_bfs`` (list-valued levels, ``seen`` a set filled
    in discovery order; networkx 3.4.2 made the pinning golden, tests/golden/e2e_pp_small.meta.json).
    networkx 2.x fills the component from set-valued levels, so CPython's set iteration order and
    with it ``Node.mask_list`` / ``point_ids`` order differ: the replay reproduces a reference run
    on networkx >= 3.0 only (the sets themselves are version-independent)."""
    level = [(n.mask_list, n.point_ids, n.node_info) for n in nodes]
    tt, aa, bb = edges
    bounds = np.searchsorted(tt, np.arange(T + 1))
    out = None
    for t in range(T):
        N = int(sizes[t])
        a, b = aa[bounds[t]:bounds[t + 1]], bb[bounds[t]:bounds[t + 1]]
        src, dst = np.concatenate([a, b]), np.concatenate([b, a])
        order = np.lexsort((dst, src))
        off = np.zeros(N + 1, np.int64)
        np.cumsum(np.bincount(src, minlength=N), out=off[1:])
        nbr = dst[order].tolist()
        adj = [nbr[off[v]:off[v + 1]] for v in range(N)]
        seen = bytearray(N)
        comps = []
        for v in range(N):                       # nx.connected_components: `for v in G`
            if seen[v]:
                continue
            c = {v}                              # _plain_bfs
            nextlevel = [v]
            while nextlevel:
                thislevel = nextlevel
                nextlevel = []
                for u in thislevel:
                    for w in adj[u]:
                        if w not in c:
                            c.add(w)
                            nextlevel.append(w)
            for u in c:
                seen[u] = 1
            comps.append(c)
        lab = np.empty(N, np.int64)
        for k, c in enumerate(comps):
            lab[list(c)] = k
        if not np.array_equal(lab, parts[t]):
            raise RuntimeError(f"replay: components of iteration {t} differ from the device's")
        new = []
        for k, c in enumerate(comps):            # Node.create_node_from_list (graph/node.py:24-37)
            mask_list = []
            point_ids = set()
            son_node_info = set()
            for i in c:
                ml, pts, info = level[i]
                mask_list += ml
                point_ids = point_ids.union(pts)
                son_node_info.add(info)
            new.append((mask_list, point_ids, (t + 1, k), son_node_info))
        level = [(m, p, i) for m, p, i, _ in new]
        out = [(m, p, s) for m, p, _, s in new]
    return out


def _level0_sequences(h):
    """(node_start, node_len, pts) of the level-0 nodes of device graph h: node i's point set as the
    reference made it, set(ascending scene ids) (utils/mask_backprojection.py:147, aliased by
    init_nodes), is pts[node_start[i] : node_start[i] + node_len[i]] (rows of the mask CSR, not
    copied); None when the mapping or a materialised set changed since construction (unknown
    history)."""
    src, node0 = h.src, h.node0
    mpc = src.mpc
    csr = getattr(mpc, "csr", None)
    if csr is None or node0 is None:
        return None
    row_of, off, pts = csr
    rows = np.fromiter((row_of[src.keys[g]] for g in node0.tolist()), np.int64, count=len(node0))
    lens = off[rows + 1] - off[rows]
    made = getattr(mpc, "_made", {})
    for k, v in made.items():                     # a set read (and maybe changed in place) by the caller
        r = row_of[k]
        row = pts[off[r]:off[r + 1]]
        if len(v) != len(row):
            return None
        # same length: the same ids in the same iteration order as the set(ascending ids) the replay
        # builds, else the caller's history (a remove and an add, say) decides the order: Python replay
        if list(v) != list(set(np.asarray(row).tolist())):
            return None
    return off[rows], lens, np.asarray(pts)


def _edge_levels(edges, T):
    tt, aa, bb = edges
    return np.searchsorted(tt, np.arange(T + 1)).astype(np.int64), aa, bb


def iterative_clustering(nodes, observer_num_thresholds, connect_threshold, debug, replay=None):
    with no_gc():
        return _iterative_clustering(nodes, observer_num_thresholds, connect_threshold, debug, replay)


def _iterative_clustering(nodes, observer_num_thresholds, connect_threshold, debug, replay):
    replay = REPLAY_SET_ORDER if replay is None else bool(replay)
    if debug:
        print('====> Start iterative clustering')
    if len(observer_num_thresholds) == 0:
        return nodes
    if len(nodes) == 0:
        raise RuntimeError("stack expects a non-empty TensorList")  # torch.stack([]) (:17)
    ctx = _device.context()
    h = _fast_path(nodes)
    if h is not None:
        F, M = h.num_frames, h.num_masks
    else:
        from . import construction
        construction._current["token"] = None  # set_nodes replaces the device graph's nodes
        F, M = _pack(ctx, nodes)
    thr = np.array([float(t) for t in observer_num_thresholds], np.float32)
    seqs = _level0_sequences(h) if (replay and h is not None) else None
    # the level-0 sets are built on a native background thread while the device clusters
    sorder = _native.SetOrder(*seqs) if seqs is not None else None
    if replay:
        cap = _EDGE_CAP0
        while True:
            ctx.set_edge_capture(cap)
            ctx.cluster(thr, connect_threshold)
            n = int(sum(ctx.edge_counts(ctx.cluster_info().num_iterations)))
            if n <= cap:
                break
            cap = n  # S6 re-runs on the same level-0 nodes with room for every edge
        edges = ctx.edges()
        ctx.set_edge_capture(0)
    else:
        ctx.cluster(thr, connect_threshold)
    ci = ctx.cluster_info()
    T = ci.num_iterations
    sizes = ctx.level_sizes(T)
    if debug:
        for t in range(T):
            print(f'Iterate {t}: observer_num', observer_num_thresholds[t], ', number of nodes', int(sizes[t]))
    obj = ctx.objects(ci, F)
    last = ctx.partition(T - 1, int(sizes[T - 1]))
    vf = bits_to_bool(obj["vf_bits"], F)
    if sorder is not None:
        # native restatement of the reference's container building (mc_setorder_begin / finish)
        eo, ea, eb = _edge_levels(edges, T)
        so = sorder.finish(sizes[:T], eo, ea, eb, labels=True)
        lab = so["labels"]
        base = 0
        for t in range(T):
            if not np.array_equal(lab[base:base + int(sizes[t])], ctx.partition(t, int(sizes[t]))):
                raise RuntimeError(f"set-order replay: components of iteration {t} differ from the device's")
            base += int(sizes[t])
        gl, node0 = h.src.gl, h.node0
        mo, mord, po, pts, sf, sord = (so["mask_off"], so["mask_order"], so["pt_off"], so["pts"], so["son_off"],
                                       so["son_order"])
        gmask = node0[mord].tolist()
        sord = sord.tolist()
        out = []
        for k in range(len(mo) - 1):
            mask_list = [gl[g] for g in gmask[mo[k]:mo[k + 1]]]
            sons = {(T - 1, j) for j in sord[sf[k]:sf[k + 1]]}      # son_node_info.add in member order
            out.append(Node.compact_lazy_points(mask_list, vf[k], obj["c_idx"][obj["c_off"][k]:obj["c_off"][k + 1]], M,
                                                pts[po[k]:po[k + 1]], (T, k), sons, ordered=True))
        return out
    if replay:
        parts = [ctx.partition(t, int(sizes[t])) for t in range(T)]
        rep = _replay(nodes, T, sizes, edges, parts)
        return [Node.compact(ml, vf[k], obj["c_idx"][obj["c_off"][k]:obj["c_off"][k + 1]], M, pts, (T, k), sons)
                for k, (ml, pts, sons) in enumerate(rep)]
    out = []
    son_order = np.argsort(last, kind="stable")                   # last-level nodes grouped by object
    son_off = np.searchsorted(last[son_order], np.arange(ci.num_objects + 1))
    son_ids = son_order.tolist()
    for k in range(ci.num_objects):
        members = obj["mask_idx"][obj["mask_off"][k]:obj["mask_off"][k + 1]]
        mask_list = []
        for i in members.tolist():
            mask_list += level0_masks(nodes[i])
        sons = {(T - 1, j) for j in son_ids[son_off[k]:son_off[k + 1]]}
        out.append(Node.compact_lazy_points(mask_list, vf[k], obj["c_idx"][obj["c_off"][k]:obj["c_off"][k + 1]], M,
                                            obj["pt_idx"][obj["pt_off"][k]:obj["pt_off"][k + 1]], (T, k), sons))
    return out
