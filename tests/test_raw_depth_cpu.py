"""The optional get_depth_raw hook of the main.py path (graph/construction.py:_raw_depth_scale,
INTEGRATION.md §2): host logic only (the device decode is tests/test_gpu_s1.py's raw-depth test)."""
import numpy as np
import pytest

from maskclustering_amd.graph import construction


class _Ds:
    depth_scale = 1000.0

    def __init__(self, raw=True, dtype=np.uint16):
        self.d = np.array([[0, 1, 999, 65535]], dtype)
        if raw:
            self.get_depth_raw = lambda f: self.d

    def get_depth(self, f):
        return (self.d / self.depth_scale).astype(np.float32)  # dataset/scannet.py:51-53

    def get_segmentation(self, f, align_with_depth=False):
        return np.zeros(self.d.shape, np.uint8)

    def get_intrinsics(self, f):
        class K:
            def get_focal_length(self):
                return (1.0, 1.0)

            def get_principal_point(self):
                return (0.0, 0.0)
        return K()

    def get_extrinsic(self, f):
        return np.eye(4)


def test_hook_selects_raw_frames(monkeypatch):
    ds = _Ds()
    assert construction._raw_depth_scale(ds) == 1000.0
    depth, seg, K, T = construction._read_frames([0, 1], ds, 1000.0)
    assert depth[0].dtype == np.uint16 and len(depth) == 2
    monkeypatch.setenv("MASKCLUSTERING_RAW_DEPTH", "0")
    assert construction._raw_depth_scale(ds) is None


def test_no_hook_reads_get_depth():
    ds = _Ds(raw=False)
    assert construction._raw_depth_scale(ds) is None
    depth, _, _, _ = construction._read_frames([0], ds, None)
    assert depth[0].dtype == np.float32


def test_hook_must_return_uint16():
    with pytest.raises(TypeError):
        construction._read_frames([0], _Ds(dtype=np.int32), 1000.0)


def test_device_decode_rule_equals_get_depth_for_every_uint16():
    """float32(u16 / scale) in float64 -- k_frames_decode's rule -- against get_depth's array for
    every uint16 value at the reference datasets' scales (1000: scannet / scannetpp / demo, 4000:
    matterport)."""
    q = np.arange(65536, dtype=np.uint16)
    for scale in (1000.0, 4000.0):
        want = (q / scale).astype(np.float32)
        got = (q.astype(np.float64) / np.float64(scale)).astype(np.float32)
        np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))
