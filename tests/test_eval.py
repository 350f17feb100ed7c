"""Instance-evaluation match lists (maskclustering_amd.evaluation.evaluate, mc_eval_match_counts)
against the reference's own assign_instances_for_scan (tests/golden/eval_small.npz, made by
tests/golden/make_eval_golden.py).  CPU: the ground-truth instance lists; GPU: the full match
structures, compared as parsed JSON (order of every list kept)."""
import json
import os
from types import SimpleNamespace

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden", "eval_small.npz")


def _ev(z, no_class):
    ids = [int(x) for x in z["class_ids"]]
    labels = [str(x) for x in z["class_labels"]]
    opt = SimpleNamespace(no_class=bool(no_class), min_region_sizes=np.array([100]))
    return SimpleNamespace(opt=opt, VALID_CLASS_IDS=ids, CLASS_LABELS=labels,
                           ID_TO_LABEL={i: l for i, l in zip(ids, labels)})


def _norm(x):
    def conv(o):
        if isinstance(o, np.integer):
            return int(o)
        if isinstance(o, np.floating):
            return float(o)
        raise TypeError(type(o))
    return json.loads(json.dumps(x, default=conv))


@pytest.mark.parametrize("seed", [0, 1])
def test_gt_instances_match_reference(seed):
    from maskclustering_amd.evaluation.evaluate import get_instances
    z = np.load(GOLD)
    c = f"s{seed}_"
    ev = _ev(z, z[c + "no_class"])
    gt = z[c + "gt"].astype(np.float64)                      # np.loadtxt gives float64 (:262)
    if ev.opt.no_class:
        gt = gt % 1000 + ev.VALID_CLASS_IDS[0] * 1000
    got = get_instances(gt, ev.VALID_CLASS_IDS, ev.CLASS_LABELS, ev.ID_TO_LABEL)
    want = json.loads(str(z[c + "gt2pred"]))
    for label in want:
        for g in want[label]:
            g.pop("matched_pred")
    assert _norm(got) == want


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [0, 1])
def test_match_lists_match_reference(seed, tmp_path):
    from maskclustering_amd.evaluation.evaluate import assign_instances_for_scan
    z = np.load(GOLD)
    c = f"s{seed}_"
    np.savetxt(tmp_path / "scene.txt", z[c + "gt"], fmt="%d")
    np.savez(tmp_path / "scene.npz", pred_masks=z[c + "pred"], pred_score=z[c + "scores"],
             pred_classes=z[c + "classes"])
    g2p, p2g = assign_instances_for_scan(str(tmp_path / "scene.npz"), str(tmp_path / "scene.txt"),
                                         _ev(z, z[c + "no_class"]))
    assert _norm(g2p) == json.loads(str(z[c + "gt2pred"]))
    assert _norm(p2g) == json.loads(str(z[c + "pred2gt"]))
