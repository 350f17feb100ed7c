"""CPU restatement of the frame decode (TEST INFRASTRUCTURE ONLY; only tests/ import it).

* depth: ``depth / depth_scale`` on the uint16 PNG values in float64, then float32
  (dataset/scannet.py:52-53; matterport.py:92, scannetpp.py:169);
* segmentation: ``cv2.resize(seg, (W, H), interpolation=cv2.INTER_NEAREST)``
  (dataset/scannet.py:72), restated as OpenCV's resizeNN index tables: source column
  ``min(floor(x * (1 / (W / Ws))), Ws - 1)``, rows alike.  cv2 is not in this container, so the
  resize is **parity unpinned** (DESIGN.md §2.2); the division is numpy's own.
"""
from __future__ import annotations

import numpy as np


def decode_depth(depth_u16, depth_scale):
    return (np.asarray(depth_u16) / depth_scale).astype(np.float32)


def nearest_tables(H, W, Hs, Ws):
    ify, ifx = 1.0 / (H / Hs), 1.0 / (W / Ws)
    yo = np.minimum(np.floor(np.arange(H) * ify).astype(np.int64), Hs - 1)
    xo = np.minimum(np.floor(np.arange(W) * ifx).astype(np.int64), Ws - 1)
    return yo, xo


def resize_nearest(seg, H, W):
    seg = np.asarray(seg)
    yo, xo = nearest_tables(H, W, seg.shape[-2], seg.shape[-1])
    return seg[..., yo, :][..., xo]
