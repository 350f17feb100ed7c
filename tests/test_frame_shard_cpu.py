"""Frame sharding on the CPU: slice arithmetic and the all-gather of
per-rank mask CSRs over gloo, world_size 2 and 3, against the single-process mask list."""
import numpy as np
import pytest

from shard_util import run_ranks


def test_frame_slices_cover_frames_in_order():
    from maskclustering_amd.frame_shard import frame_slice
    for F in (0, 1, 2, 7, 250, 1501):
        for world in (1, 2, 3, 4, 8, 16):
            sl = [frame_slice(F, world, r) for r in range(world)]
            assert sl[0][0] == 0 and sl[-1][1] == F
            assert all(a[1] == b[0] for a, b in zip(sl, sl[1:]))
            sizes = [hi - lo for lo, hi in sl]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        frame_slice(10, 2, 2)


@pytest.mark.parametrize("world", [2, 3])
def test_gather_equals_global_mask_list(tmp_path, world):
    from maskclustering_amd.synthetic import make_shape
    s = make_shape("tiny", seed=4)
    for out in run_ranks("gather", world, tmp_path):
        z = np.load(out)
        np.testing.assert_array_equal(z["col"], s.mask_col)
        np.testing.assert_array_equal(z["label"], s.mask_label)
        np.testing.assert_array_equal(z["off"], s.mask_off)
        np.testing.assert_array_equal(z["pts"], s.mask_pts)
