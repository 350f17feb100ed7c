"""Instance evaluation with the match counts on the device.

The reference's ``evaluation/evaluate.py`` parses its command line at import and keeps the
label tables in module globals; ``assign_instances_for_scan`` (:254-329) builds, per scan, the
gt -> prediction and prediction -> gt match lists from one bool column product per predicted
mask (:308, on the GPU through torch).  Here that product, the vertex counts and the void
intersections of all masks of a scan are one C-ABI call (``mc_eval_match_counts``: a per-point
histogram over the [P, K] prediction matrix), and the match lists are rebuilt exactly as the
reference builds them (same dict layout, order and number types).  AP (``evaluate_matches``
:53-205) and the reports stay the reference's.

Run from the reference's root instead of ``python -m evaluation.evaluate ...``:

    python -m maskclustering_amd.evaluation.evaluate --pred_path ... --gt_path ... --dataset scannet [--no_class]

which imports the reference's module (its argument parsing and tables), routes its
``assign_instances_for_scan`` here and runs its ``main``.
"""
from __future__ import annotations

import os
import sys
from copy import deepcopy

import numpy as np

from .. import _device


def get_instances(ids, class_ids, class_labels, id2label):
    """evaluation/utils_3d.py:53-65: ground-truth instances per label (instance id = label * 1000 + k,
    0 = none), each as the dict Instance.to_dict gives (:36-43)."""
    out = {label: [] for label in class_labels}
    uniq, counts = np.unique(ids, return_counts=True)
    for iid, cnt in zip(uniq.tolist(), counts.tolist()):
        if iid == 0:
            continue
        label_id = int(int(iid) // 1000)
        if label_id in class_ids:
            out[id2label[label_id]].append({"instance_id": int(iid), "label_id": label_id, "vert_count": int(cnt),
                                            "med_dist": -1, "dist_conf": 0.0})
    return out


def assign_instances_for_scan(pred_file, gt_file, ev=None):
    """evaluation/evaluate.py:254-329.  ``ev`` holds the reference module's globals (opt,
    VALID_CLASS_IDS, CLASS_LABELS, ID_TO_LABEL); default: the imported reference module."""
    if ev is None:
        ev = sys.modules["evaluation.evaluate"]
    opt = ev.opt
    pred = np.load(os.path.join(pred_file))                     # read_pridiction_npz (:226-238)
    base = pred_file.split('/')[-1]
    masks, scores, classes = pred['pred_masks'], pred['pred_score'], pred['pred_classes']
    gt_ids = np.loadtxt(gt_file)
    if opt.no_class:
        gt_ids = gt_ids % 1000 + ev.VALID_CLASS_IDS[0] * 1000
    gt_instances = get_instances(gt_ids, ev.VALID_CLASS_IDS, ev.CLASS_LABELS, ev.ID_TO_LABEL)
    gt2pred = deepcopy(gt_instances)
    for label in gt2pred:
        for gt in gt2pred[label]:
            gt['matched_pred'] = []
    pred2gt = {label: [] for label in ev.CLASS_LABELS}
    bool_void = np.logical_not(np.isin(gt_ids // 1000, ev.VALID_CLASS_IDS))  # np.in1d at :273
    # every point's instance as one global index: the labels' instance lists back to back
    first, ginst, G = {}, np.full(len(gt_ids), -1, np.int32), 0
    for label, insts in gt_instances.items():
        first[label] = G
        for inst in insts:
            ginst[gt_ids == inst['instance_id']] = G
            G += 1
    K = len(scores)
    if masks.shape[0] == len(gt_ids) and K:
        verts, vint, inter = _device.context().eval_match_counts(masks, ginst, G, bool_void)
    num_pred_instances = 0
    for i in range(K):
        label_id = ev.VALID_CLASS_IDS[0] if opt.no_class else int(classes[i])
        conf = scores[i]
        if label_id not in ev.ID_TO_LABEL:
            continue
        label_name = ev.ID_TO_LABEL[label_id]
        if masks.shape[0] != len(gt_ids):
            print('wrong number of lines in ' + f"{base}_{i}" + '(%d) vs #mesh vertices (%d), please double check '
                  'and/or re-download the mesh' % (masks.shape[0], len(gt_ids)))
            raise NotImplementedError
        num = int(verts[i])
        if num < opt.min_region_sizes[0]:
            continue
        pred_instance = {'filename': f"{base}_{i}", 'pred_id': num_pred_instances, 'label_id': label_id,
                         'vert_count': num, 'confidence': conf, 'void_intersection': int(vint[i])}
        matched_gt = []
        g0, n = first[label_name], len(gt_instances[label_name])
        row = inter[i, g0:g0 + n]
        for gt_id in np.nonzero(row)[0].tolist():
            gt_copy = gt_instances[label_name][gt_id].copy()
            pred_copy = pred_instance.copy()
            gt_copy['intersection'] = int(row[gt_id])
            pred_copy['intersection'] = int(row[gt_id])
            matched_gt.append(gt_copy)
            gt2pred[label_name][gt_id]['matched_pred'].append(pred_copy)
        pred_instance['matched_gt'] = matched_gt
        num_pred_instances += 1
        pred2gt[label_name].append(pred_instance)
    return gt2pred, pred2gt


def main():
    import importlib
    ev = importlib.import_module("evaluation.evaluate")        # the reference's: parses sys.argv
    ev.assign_instances_for_scan = lambda pred_file, gt_file: assign_instances_for_scan(pred_file, gt_file, ev)
    ev.main()


if __name__ == "__main__":
    main()
