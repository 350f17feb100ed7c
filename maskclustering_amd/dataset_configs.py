"""The graph path's thresholds per dataset, as the reference's `configs/*.json` hold them, and the
dataset config each synthetic shape stands in for (C1 demo, C2 ScanNet, C3 ScanNet++,
C4 Matterport3D).

The four keys are the ones the graph path reads (`graph/construction.py:119,125,132` and
`main.py:19`); `point_filter_threshold` is post_process's (`utils/post_process.py:173`).  ScanNet++
is the config whose edge rule differs: view_consensus_threshold = 1 gives smin[1] = 2, so pairs
observed together in one frame never connect."""
from __future__ import annotations

# configs/<name>.json:2-6 of the reference
DATASET_THRESHOLDS = {
    "demo": dict(mask_visible_threshold=0.3, undersegment_filter_threshold=0.3, view_consensus_threshold=0.9,
                 contained_threshold=0.8, point_filter_threshold=0.5),
    "scannet": dict(mask_visible_threshold=0.3, undersegment_filter_threshold=0.3, view_consensus_threshold=0.9,
                    contained_threshold=0.8, point_filter_threshold=0.5),
    "scannetpp": dict(mask_visible_threshold=0.4, undersegment_filter_threshold=0.2, view_consensus_threshold=1,
                      contained_threshold=0.9, point_filter_threshold=0.7),
    "matterport3d": dict(mask_visible_threshold=0.3, undersegment_filter_threshold=0.3, view_consensus_threshold=0.9,
                         contained_threshold=0.8, point_filter_threshold=0.5),
    "tasmap": dict(mask_visible_threshold=0.2, undersegment_filter_threshold=0.1, view_consensus_threshold=0.9,
                   contained_threshold=0.8, point_filter_threshold=0.5),
}

# the dataset config each synthetic shape is measured and tested under (BASELINE.json configs[0..3])
SHAPE_DATASET = {"few": "scannet", "tiny": "scannet", "c1": "demo", "c2": "scannet", "c2x2": "scannet",
                 "c3": "scannetpp", "c4": "matterport3d"}

GRAPH_KEYS = ("mask_visible_threshold", "undersegment_filter_threshold", "view_consensus_threshold",
              "contained_threshold")


def graph_thresholds(dataset: str) -> dict:
    """the four thresholds GraphRun.step / the oracle's run take, for dataset config `dataset`"""
    t = DATASET_THRESHOLDS[dataset]
    return {k: t[k] for k in GRAPH_KEYS}


def shape_thresholds(shape: str) -> tuple[str, dict]:
    """(dataset config name, graph thresholds) of a synthetic shape"""
    ds = SHAPE_DATASET.get(shape, "scannet")
    return ds, graph_thresholds(ds)
