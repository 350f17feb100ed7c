"""Frame decode (maskclustering_amd.scene_pack, mc_frames_decode) against the CPU restatement
(oracle/io_oracle.py).  The nearest-neighbour resize is parity unpinned (cv2 absent): the CPU
tests pin the restatement's index tables on known answers."""
import numpy as np
import pytest

from oracle import io_oracle


def test_nearest_tables_known_answers():
    yo, xo = io_oracle.nearest_tables(480, 640, 480, 640)
    assert (yo == np.arange(480)).all() and (xo == np.arange(640)).all()          # same size: identity
    yo, xo = io_oracle.nearest_tables(240, 320, 480, 640)
    assert (yo == 2 * np.arange(240)).all() and (xo == 2 * np.arange(320)).all()  # 2x down: even rows / columns
    yo, xo = io_oracle.nearest_tables(480, 640, 240, 320)
    assert (xo == np.arange(640) // 2).all()                                      # 2x up: repeats
    yo, xo = io_oracle.nearest_tables(480, 640, 968, 1296)                         # ScanNet colour -> depth
    assert xo[0] == 0 and xo[1] == 2 and xo[639] == 1293 and yo[479] == 965 and xo.max() < 1296


def test_depth_division_is_float64_then_float32():
    d = np.array([[1, 999, 1001, 65535]], np.uint16)
    got = io_oracle.decode_depth(d, 1000.0)
    assert got.dtype == np.float32
    assert got.tolist() == [[np.float32(1 / 1000.0), np.float32(999 / 1000.0), np.float32(1001 / 1000.0),
                             np.float32(65535 / 1000.0)]]


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [((4, 480, 640), (968, 1296), 1000.0), ((3, 240, 320), (240, 320), 4000.0),
                                   ((2, 480, 640), (240, 320), 1000.0), ((2, 37, 53), (101, 13), 1000.0)])
def test_decode_matches_oracle(shape, tmp_path):
    from maskclustering_amd.scene_pack import decode_frames, load_scene_pack, write_scene_pack
    (F, H, W), (Hs, Ws), scale = shape
    rng = np.random.default_rng(F * H)
    depth = rng.integers(0, 65536, (F, H, W)).astype(np.uint16)
    seg = rng.integers(0, 256, (F, Hs, Ws)).astype(np.uint8)
    d, s = decode_frames(depth, seg, scale)
    np.testing.assert_array_equal(d.cpu().numpy(), io_oracle.decode_depth(depth, scale))
    np.testing.assert_array_equal(s.cpu().numpy(), io_oracle.resize_nearest(seg, H, W))
    p = tmp_path / "scene.npz"
    write_scene_pack(p, depth, seg, np.tile([500.0, 500.0, W / 2, H / 2], (F, 1)), np.tile(np.eye(4), (F, 1, 1)),
                     list(range(0, 10 * F, 10)), scale)
    z = load_scene_pack(p)
    np.testing.assert_array_equal(z["depth"].cpu().numpy(), d.cpu().numpy())
    np.testing.assert_array_equal(z["seg"].cpu().numpy(), s.cpu().numpy())
    assert z["frame_ids"] == list(range(0, 10 * F, 10))
