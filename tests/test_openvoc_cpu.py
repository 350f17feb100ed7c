"""Open-vocabulary query: the CPU restatement against the reference's own
main() output (tests/golden/openvoc_small.npz, made by tests/golden/make_openvoc_golden.py)."""
import os

import numpy as np

from oracle import openvoc_oracle

GOLD = os.path.join(os.path.dirname(__file__), "golden", "openvoc_small.npz")


def load():
    return dict(np.load(GOLD))


def test_oracle_matches_reference_main():
    z = load()
    lab, _ = openvoc_oracle.query(z["obj_off"], z["obj_rows"], z["feats"].astype(np.float32),
                                  z["labels"].astype(np.float32))
    ids = z["label_ids"]
    want = z["pred_classes"]
    got = np.where(lab >= 0, ids[np.maximum(lab, 0)], 0)
    np.testing.assert_array_equal(got, want)
    # the fixture covers the empty, exact-tie and overflow (NaN) cases
    assert (lab < 0).sum() >= 3
    assert lab[4] == 5                      # labels 5 and 17 are equal: the first wins
    assert lab[3] == 40                     # feature == label 40: exp overflow, the first NaN
