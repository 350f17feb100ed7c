"""CPU restatement of the reference's open-vocabulary label query (TEST INFRASTRUCTURE ONLY).

Only ``tests/`` may import this module, as the checker of the HIP path
(``maskclustering_amd.semantics.open_voc_query``); the product never routes through it.

Restates ``semantics/open-voc_query.py:32-53`` in numpy, operation for operation: per object
with a representative mask, the float32 mean of its masks' features (np.mean over axis 0),
``np.dot`` with the label text features, ``np.exp(sim * 100)``, the softmax row and
``np.argmax(np.max(prob, axis=0))`` (first maximum; the first NaN when exp overflowed).  Also
returns the probability rows, which the GPU test uses to tell a genuine mismatch from a
float32-ULP near-tie (the device sums the dot products in another order).  Pinned by
``tests/golden/openvoc_small.npz`` (the reference's own main(), tests/test_openvoc_cpu.py).
"""
from __future__ import annotations

import numpy as np


def query(obj_off, obj_rows, feats, label_feats, temperature=100):
    """-> (label index per object, -1 for objects with no representative mask; prob rows)"""
    labels, probs = [], []
    for k in range(len(obj_off) - 1):
        rows = obj_rows[obj_off[k]:obj_off[k + 1]]
        if len(rows) == 0:                                        # :33-34
            labels.append(-1)
            probs.append(None)
            continue
        feature = np.stack([feats[r] for r in rows])              # :36-38
        object_feature = np.mean(feature, axis=0, keepdims=True)  # :39
        raw = np.dot(object_feature, label_feats.T)               # :41
        with np.errstate(over="ignore", invalid="ignore"):
            exp_sim = np.exp(raw * temperature)                   # :42
            prob = exp_sim / np.sum(exp_sim, axis=1, keepdims=True)
        labels.append(int(np.argmax(np.max(prob, axis=0))))      # :44
        probs.append(prob[0])
    return np.array(labels, np.int64), probs
