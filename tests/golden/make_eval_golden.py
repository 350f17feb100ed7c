"""Golden fixtures for the evaluation match lists: the REFERENCE's own
``evaluation/evaluate.py`` ``assign_instances_for_scan`` (:254-329) on synthetic ground truth
and predictions, class-aware and ``--no_class``.

Run ONLY in the build container, where /root/reference exists:

    python tests/golden/make_eval_golden.py

The reference module is imported unmodified (its argument parsing reads the sys.argv set
here; torch's ``.cuda()`` is the identity on this CPU-only container).  The fixture holds the
inputs (gt ids, the prediction matrix, scores, classes, the scannet label table from
evaluation/constants.py) and the two match structures as JSON.  No source is copied.
"""
from __future__ import annotations

import importlib
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def to_json(x):
    def conv(o):
        if isinstance(o, np.integer):
            return int(o)
        if isinstance(o, np.floating):
            return float(o)
        raise TypeError(type(o))
    return json.dumps(x, default=conv)


def synthetic(seed, ids):
    rng = np.random.default_rng(seed)
    P, K = 6000, 48
    gt = np.zeros(P, np.int64)
    valid = list(ids)
    start = 0
    n = 0
    while start < P - 50:                      # runs of points per instance (plus unlabeled gaps)
        ln = int(rng.integers(20, 400))
        r = rng.random()
        lab = int(rng.choice(valid)) if r < 0.8 else (0 if r < 0.9 else 999)   # 999: not a class id (void)
        gt[start:start + ln] = lab * 1000 + n if lab else 0
        n += 1
        start += ln + int(rng.integers(0, 30))
    pred = np.zeros((P, K), bool)
    for k in range(K):
        a = int(rng.integers(0, P - 10))
        ln = int(rng.integers(5, 700))
        pred[a:a + ln, k] = True
        pred[rng.integers(0, P, 30), k] = True
    scores = rng.random(K)
    classes = np.array([int(rng.choice(valid)) if rng.random() < 0.85 else 999 for _ in range(K)], np.int32)
    return gt, pred, scores, classes


def run_reference(tmp, gt, pred, scores, classes, no_class):
    sys.dont_write_bytecode = True
    import torch
    torch.Tensor.cuda = lambda self, *a, **k: self
    if REF not in sys.path:
        sys.path.insert(0, REF)
    sys.argv = ["evaluate.py", "--pred_path", tmp, "--gt_path", tmp, "--dataset", "scannet"] + \
        (["--no_class"] if no_class else [])
    for m in [m for m in sys.modules if m == "evaluation.evaluate"]:
        del sys.modules[m]
    ev = importlib.import_module("evaluation.evaluate")
    np.savetxt(os.path.join(tmp, "scene.txt"), gt, fmt="%d")
    np.savez(os.path.join(tmp, "scene.npz"), pred_masks=pred, pred_score=scores, pred_classes=classes)
    g2p, p2g = ev.assign_instances_for_scan(os.path.join(tmp, "scene.npz"), os.path.join(tmp, "scene.txt"))
    return ev, g2p, p2g


def main():
    if REF not in sys.path:
        sys.path.insert(0, REF)
    from evaluation import constants
    ids = list(constants.SCANNET_IDS)
    out = {"class_ids": np.array(ids, np.int64), "class_labels": np.array(list(constants.SCANNET_LABELS))}
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as tmp:
        os.chdir(tmp)
        try:
            for seed, no_class in ((0, False), (1, True)):
                gt, pred, scores, classes = synthetic(seed, ids)
                ev, g2p, p2g = run_reference(tmp, gt, pred, scores, classes, no_class)
                c = f"s{seed}_"
                out.update({c + "gt": gt, c + "pred": pred, c + "scores": scores, c + "classes": classes,
                            c + "no_class": np.array(no_class), c + "gt2pred": np.array(to_json(g2p)),
                            c + "pred2gt": np.array(to_json(p2g))})
                print(f"seed {seed} no_class={no_class}: gt instances "
                      f"{sum(len(v) for v in g2p.values())}, preds {sum(len(v) for v in p2g.values())}, "
                      f"matches {sum(len(p['matched_gt']) for v in p2g.values() for p in v)}")
        finally:
            os.chdir(cwd)
    np.savez_compressed(os.path.join(HERE, "eval_small.npz"), **out)


if __name__ == "__main__":
    main()
