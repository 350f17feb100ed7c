"""Golden fixtures for S1 (per-frame mask back-projection) from the REFERENCE's
own glue code.

Run ONLY in the build container, where /root/reference exists:

    python tests/golden/make_s1_golden.py

``utils/mask_backprojection.py`` is imported unmodified.  Open3D and pytorch3d
are absent from this container, so the library calls it makes
are served by the small restatements below (Open3D: depth->point cloud,
transform, voxel_down_sample, cluster_dbscan, select_by_index,
remove_statistical_outlier; pytorch3d: ball_query).  They are independent of
the C oracle (numpy / Python sets, Open3D's DBSCAN loop taken literally, the
float32 FMA of the ball query emulated in long double), so a fixture pins:

* the reference's glue, exactly: id order (torch.unique + sort), the depth
  mask vs point-cloud alignment, FEW_POINTS_THRESHOLD twice, float32 casts,
  crop_scene_points (the reference's own torch code), padding + lengths of the
  batched ball query, torch.unique of the neighbours, coverage, set unions;
* the library semantics only as restated (parity unpinned there: DESIGN.md §5).

Outputs are data (inputs and the reference's outputs); no source is copied.
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"


# ------------------------------------------------------------------------------------------
# restated library ops (stubs for the absent modules)
# ------------------------------------------------------------------------------------------
class _Image:
    def __init__(self, arr):
        self.arr = np.asarray(arr)


class _Intrinsic:
    def __init__(self, fx, fy, cx, cy):
        self.fx, self.fy, self.cx, self.cy = float(fx), float(fy), float(cx), float(cy)


def _d2(a, b):
    d = a[None, :, :] - b[:, None, :] if False else a[:, None, :] - b[None, :, :]
    return (d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2]


class _PointCloud:
    def __init__(self, pts=None):
        self.points = np.zeros((0, 3)) if pts is None else np.asarray(pts, np.float64).reshape(-1, 3)

    @staticmethod
    def create_from_depth_image(depth, intr, depth_scale=1.0, depth_trunc=1000.0, **kw):
        d = depth.arr.astype(np.float32) / np.float32(depth_scale)
        d = np.where(d.astype(np.float64) >= depth_trunc, np.float32(0), d)
        v, u = np.nonzero(d > 0)                       # row-major
        z = d[v, u].astype(np.float64)
        x = (u.astype(np.float64) - intr.cx) * z / intr.fx
        y = (v.astype(np.float64) - intr.cy) * z / intr.fy
        return _PointCloud(np.stack([x, y, z], axis=1))

    def transform(self, T):
        T = np.asarray(T, np.float64)
        p = self.points
        r = [((T[k, 0] * p[:, 0] + T[k, 1] * p[:, 1]) + T[k, 2] * p[:, 2]) + T[k, 3] for k in range(4)]
        self.points = np.stack([r[0] / r[3], r[1] / r[3], r[2] / r[3]], axis=1)
        return self

    def voxel_down_sample(self, voxel_size):
        p = self.points
        vmin = p.min(axis=0) - voxel_size * 0.5
        idx = np.floor((p - vmin) / voxel_size).astype(np.int64)
        acc = {}
        for i in range(len(p)):
            k = tuple(idx[i])
            if k not in acc:
                acc[k] = [np.zeros(3), 0]
            s = acc[k]
            s[0] = s[0] + p[i]   # sequential sum in input order
            s[1] += 1
        return _PointCloud(np.array([s / float(c) for s, c in acc.values()]).reshape(-1, 3))

    def cluster_dbscan(self, eps, min_points, print_progress=False):
        p = self.points
        n = len(p)
        nbs = [np.nonzero(row < eps * eps)[0].tolist() for row in _d2(p, p)]
        labels = [-2] * n
        cl = 0
        for idx in range(n):          # Open3D ClusterDBSCAN, with Python sets as its unordered_set
            if labels[idx] != -2:
                continue
            if len(nbs[idx]) < min_points:
                labels[idx] = -1
                continue
            nxt = set(nbs[idx])
            visited = {idx}
            labels[idx] = cl
            while nxt:
                nb = nxt.pop()
                visited.add(nb)
                if labels[nb] == -1:
                    labels[nb] = cl
                if labels[nb] != -2:
                    continue
                labels[nb] = cl
                if len(nbs[nb]) >= min_points:
                    for q in nbs[nb]:
                        if q not in visited:
                            nxt.add(q)
            cl += 1
        return types.SimpleNamespace(__array__=None) if False else labels

    def select_by_index(self, idx):
        return _PointCloud(self.points[np.asarray(idx, np.int64)])

    def remove_statistical_outlier(self, nb_neighbors, std_ratio):
        p = self.points
        m = len(p)
        if m == 0:
            return _PointCloud(), []
        kk = min(nb_neighbors, m)
        d = np.sort(_d2(p, p), axis=1)[:, :kk]
        avg = np.zeros(m)
        for i in range(m):
            s = 0.0
            for j in range(kk):
                s += float(np.sqrt(d[i, j]))
            avg[i] = s / kk
        mean = 0.0
        for a in avg:
            if a > 0:
                mean += a
        mean /= m
        sq = 0.0
        for a in avg:
            sq += (a - mean) * (a - mean) if a > 0 else 0.0
        with np.errstate(divide="ignore", invalid="ignore"):
            thr = mean + std_ratio * np.sqrt(np.float64(sq) / np.float64(m - 1))
        keep = [i for i in range(m) if avg[i] > 0 and avg[i] < thr]
        return _PointCloud(p[keep]), keep


def _ball_query(p1, p2, lengths1=None, lengths2=None, K=500, radius=0.2, return_nn=True):
    """pytorch3d 0.7.3 ball_query (CUDA kernel semantics, nvcc FMA contraction)."""
    import torch
    P1 = p1.detach().cpu().numpy().astype(np.float32)
    P2 = p2.detach().cpu().numpy().astype(np.float32)
    l1 = lengths1.cpu().numpy()
    l2 = lengths2.cpu().numpy()
    r = np.float32(radius)
    r2 = np.float32(r * r)
    N, S1 = P1.shape[:2]
    idx = -np.ones((N, S1, K), np.int64)
    for n in range(N):
        q = P1[n, :l1[n]]
        s = P2[n, :l2[n]]
        for i in range(len(q)):
            dx = (q[i, 0] - s[:, 0]).astype(np.float32)
            dy = (q[i, 1] - s[:, 1]).astype(np.float32)
            dz = (q[i, 2] - s[:, 2]).astype(np.float32)
            xx = (dx * dx).astype(np.float32)
            t = (dy.astype(np.longdouble) * dy + xx).astype(np.float32)      # fmaf(dy, dy, xx)
            d2 = (dz.astype(np.longdouble) * dz + t).astype(np.float32)      # fmaf(dz, dz, t)
            hit = np.nonzero(d2 < r2)[0][:K]
            idx[n, i, :len(hit)] = hit
    return None, torch.from_numpy(idx), None


def _import_reference():
    sys.dont_write_bytecode = True
    import torch
    o3d = types.ModuleType("open3d")
    o3d.geometry = types.SimpleNamespace(Image=_Image, PointCloud=_PointCloud)
    o3d.utility = types.SimpleNamespace(Vector3dVector=lambda a: np.asarray(a, np.float64))
    o3d.camera = types.SimpleNamespace(PinholeCameraIntrinsic=_Intrinsic)
    sys.modules["open3d"] = o3d
    p3d = types.ModuleType("pytorch3d")
    ops = types.ModuleType("pytorch3d.ops")
    ops.ball_query = _ball_query
    sys.modules["pytorch3d"] = p3d
    sys.modules["pytorch3d.ops"] = ops
    sys.modules.setdefault("cv2", types.ModuleType("cv2"))
    torch.Tensor.cuda = lambda self, *a, **k: self
    if REF not in sys.path:
        sys.path.insert(0, REF)
    from utils import mask_backprojection  # noqa: E402
    return mask_backprojection, torch


class _Dataset:
    """The four dataset methods turn_mask_to_point reads (mask_backprojection.py:71-72,80)."""

    def __init__(self, frames):
        self.fr = frames

    def get_intrinsics(self, f):
        fx, fy, cx, cy = self.fr.intrinsics[f]
        return _Intrinsic(fx, fy, cx, cy)

    def get_extrinsic(self, f):
        return self.fr.poses[f].copy()

    def get_depth(self, f):
        return self.fr.depth[f].copy()


def run_reference_frames(frames):
    mb, torch = _import_reference()
    ds = _Dataset(frames)
    scene = torch.tensor(frames.scene_points).float()          # construction.py:37
    out_labels, out_off, out_pts, out_err = [], [0], [], []
    frame_off = [0]
    for f in range(frames.num_frames):
        try:
            info, valid, fpts = mb.turn_mask_to_point(ds, scene, frames.seg[f].copy(), f)
            err = 0
        except IndexError:
            info, valid, fpts, err = {}, [], [], 1
        out_err.append(err)
        for mid in sorted(info):
            out_labels.append(int(mid))
            s = np.array(sorted(int(x) for x in info[mid]), np.int32)
            out_pts.append(s)
            out_off.append(out_off[-1] + len(s))
        frame_off.append(len(out_labels))
        assert sorted(int(m) for m in info) == sorted(int(m) for m in valid)
        assert sorted(int(x) for x in fpts) == sorted(set().union(*[set(int(y) for y in v) for v in info.values()]))
    return dict(out_labels=np.array(out_labels, np.int32), out_off=np.array(out_off, np.int64),
                out_pts=np.concatenate(out_pts).astype(np.int32) if out_pts else np.zeros(0, np.int32),
                out_frame_off=np.array(frame_off, np.int64), out_err=np.array(out_err, np.int32))


def edge_frames():
    """A small scene with the reference's edge cases: an inf pose (:73-74), a
    frame with no mask ids, a frame whose only masks are below 25 pixels, a
    DEPTH_TRUNC pixel (IndexError, :100), and a mask of depth-invalid pixels."""
    sys.path.insert(0, REPO)
    from maskclustering_amd.synthetic_frames import make_frames_shape
    fr = make_frames_shape("tiny", seed=3, H=90, W=120)
    fr.poses[1, 0, 3] = np.inf
    fr.seg[2] = 0
    fr.seg[3] = np.where(fr.seg[3] > 0, 0, 0).astype(np.uint8)
    fr.seg[3, :4, :5] = 7                       # 20 pixels only
    fr.depth[4, 0, 0] = np.float32(20.0)         # == DEPTH_TRUNC with ids present -> IndexError
    fr.seg[5, fr.depth[5] > 0] = fr.seg[5, fr.depth[5] > 0]
    fr.depth[5, 10:40, 10:60] = 0.0              # ids over invalid depth
    fr.seg[5, 10:40, 10:60] = 200
    return fr


def save(name, frames):
    ref = run_reference_frames(frames)
    inp = dict(in_scene=frames.scene_points, in_depth=frames.depth, in_seg=frames.seg,
               in_intrinsics=frames.intrinsics, in_poses=frames.poses)
    path = os.path.join(HERE, f"s1_{name}.npz")
    np.savez_compressed(path, **inp, **ref)
    print(f"s1_{name}: frames={frames.num_frames} masks={len(ref['out_labels'])} pts={len(ref['out_pts'])} "
          f"errors={ref['out_err'].tolist()} -> {os.path.getsize(path) / 1e6:.2f} MB")


def main():
    sys.path.insert(0, REPO)
    from maskclustering_amd.synthetic_frames import make_frames_shape
    save("tiny", make_frames_shape("tiny", seed=0))
    save("dense", make_frames_shape("tiny", seed=1, H=240, W=320, num_frames=4))
    save("edge", edge_frames())


if __name__ == "__main__":
    main()
