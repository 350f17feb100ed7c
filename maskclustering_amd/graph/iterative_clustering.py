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

``mask_list`` of a merged node lists its members' masks in ascending member
order and ``point_ids`` is the union set; the reference's order inside these
containers follows CPython set iteration and is not reproduced.
"""
from __future__ import annotations

import numpy as np

from .. import _device
from ..pipeline import bits_to_bool, bool_to_bits
from .node import Node


def _fast_path(nodes):
    from . import construction
    if not nodes:
        return None
    h = getattr(nodes[0], "_graph", None)
    if h is None or h.token != construction._current["token"] or len(nodes) != h.num_nodes:
        return None
    for i, n in enumerate(nodes):
        if getattr(n, "_graph", None) is not h or n._level0 != i or getattr(n, "_vf", None) is None \
                or getattr(n, "_cids", None) is None:
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


def iterative_clustering(nodes, observer_num_thresholds, connect_threshold, debug):
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
    out = []
    for k in range(ci.num_objects):
        members = obj["mask_idx"][obj["mask_off"][k]:obj["mask_off"][k + 1]]
        mask_list = []
        for i in members.tolist():
            mask_list += nodes[i].mask_list
        sons = {(T - 1, int(j)) for j in np.nonzero(last == k)[0].tolist()}
        out.append(Node.compact(mask_list, vf[k], obj["c_idx"][obj["c_off"][k]:obj["c_off"][k + 1]], M,
                                set(obj["pt_idx"][obj["pt_off"][k]:obj["pt_off"][k + 1]].tolist()), (T, k), sons))
    return out
