"""The S1 CPU restatement (oracle/s1_oracle.c) against fixtures made by running
the reference's own utils/mask_backprojection.py (tests/golden/make_s1_golden.py),
plus independent cross-checks of the restated library steps.  Parity of the
Open3D / pytorch3d arithmetic itself is unpinned."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import oracle

S1_CASES = ["s1_tiny", "s1_dense", "s1_edge"]


def _frames(z):
    from types import SimpleNamespace
    return SimpleNamespace(scene_points=z["in_scene"], depth=z["in_depth"], seg=z["in_seg"],
                           intrinsics=z["in_intrinsics"], poses=z["in_poses"], num_frames=len(z["in_depth"]))


@pytest.mark.parametrize("name", S1_CASES)
def test_s1_oracle_matches_reference_glue(name):
    z = dict(np.load(os.path.join(GOLDEN, name + ".npz")))
    fr = _frames(z)
    scene = fr.scene_points.astype(np.float32)
    fo = z["out_frame_off"]
    for f in range(fr.num_frames):
        if z["out_err"][f]:
            with pytest.raises(IndexError):
                oracle.s1_frame(scene, fr.depth[f], fr.seg[f], fr.intrinsics[f], fr.poses[f])
            continue
        lab, off, pts, st = oracle.s1_frame(scene, fr.depth[f], fr.seg[f], fr.intrinsics[f], fr.poses[f])
        g0, g1 = fo[f], fo[f + 1]
        np.testing.assert_array_equal(lab, z["out_labels"][g0:g1], err_msg=f"frame {f} labels")
        for k in range(len(lab)):
            want = z["out_pts"][z["out_off"][g0 + k]:z["out_off"][g0 + k + 1]]
            np.testing.assert_array_equal(pts[off[k]:off[k + 1]], want, err_msg=f"frame {f} mask {lab[k]}")


def test_s1_stage_counts_are_monotone():
    z = dict(np.load(os.path.join(GOLDEN, "s1_dense.npz")))
    fr = _frames(z)
    for f in range(fr.num_frames):
        _, _, _, st = oracle.s1_frame(fr.scene_points.astype(np.float32), fr.depth[f], fr.seg[f],
                                      fr.intrinsics[f], fr.poses[f])
        big = st[st[:, 1] >= 25]
        assert (big[:, 2] <= big[:, 1]).all()      # voxels <= pixels
        assert (big[:, 3] <= big[:, 2]).all()      # DBSCAN class filter
        assert (big[:, 4] <= big[:, 3]).all()      # statistical outlier removal
        kept = big[big[:, 8] == 1]
        assert (kept[:, 6] >= 0.3 * kept[:, 4]).all()  # coverage
