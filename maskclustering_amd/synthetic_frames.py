"""Synthetic RGB-D frames for the end-to-end path (S1 back-projection -> S6).

A static world of boxes on a floor is rendered analytically (ray/box slabs)
from a camera that travels along the row of boxes.  Every frame yields what the
reference's datasets return for one frame id:

* ``depth``   float32 [H,W] metres, quantised like the datasets' uint16 PNGs:
              float32(uint16 / depth_scale) computed in float64
              (``dataset/scannet.py:49-54``: 1000; ``matterport.py:89-94``: 4000,
              values past 65535 units read as 0); floor and back wall give depth
              but no mask;
* ``seg``     uint8 [H,W] instance ids 1..k ascending in object order
              (``mask_predict.py:102-113``), with occasional split masks (one
              object, two ids) and merged masks (two objects, one id);
* ``K``       fx, fy, cx, cy (``dataset/scannet.py:34-40``);
* ``pose``    4x4 camera-to-world (``dataset/scannet.py:43-46``);

and the scene points are samples of the box surfaces on a jittered grid, like
mesh vertices (``get_scene_points``, ``dataset/scannet.py:87-90``).

The renderer runs in torch float64 on the device it is given (CPU for tests,
the GPU for bench-sized scenes); it is input plumbing, not part of the path.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np


@dataclass
class SceneFrames:
    scene_points: np.ndarray  # float64 [P,3]
    depth: np.ndarray         # float32 [F,H,W]
    seg: np.ndarray           # uint8 [F,H,W]
    intrinsics: np.ndarray    # float64 [F,4]  fx, fy, cx, cy
    poses: np.ndarray         # float64 [F,4,4]
    meta: dict = field(default_factory=dict)

    @property
    def num_frames(self) -> int:
        return int(self.depth.shape[0])

    @property
    def num_points(self) -> int:
        return int(self.scene_points.shape[0])


FRAME_SHAPES = {
    # tests: seconds on the CPU oracle
    "tiny": dict(num_objects=10, num_frames=8, H=60, W=80, length=2.5, spacing=0.02, size=(0.12, 0.3)),
    "small": dict(num_objects=30, num_frames=16, H=120, W=160, length=5.0, spacing=0.02, size=(0.12, 0.3)),
    # ScanNet-shaped (BASELINE configs[1]): 640x480, 250 frames, ~240k points, ~60 masks per frame (~15k)
    "c2": dict(num_objects=760, num_frames=250, H=480, W=640, length=50.0, spacing=0.025, size=(0.1, 0.3),
               frame_rng=True),
    # the round-1 ScanNet-shaped stand-in (P 194k, M 11.8k), kept for comparisons with its profiles
    "c2_r1": dict(num_objects=600, num_frames=250, H=480, W=640, length=50.0, spacing=0.025, size=(0.1, 0.3)),
    # ScanNet++-shaped (BASELINE configs[2], dataset/scannetpp.py:126): 1920x1440, 1500 frames, ~1M points,
    # ~80k masks
    "c3": dict(num_objects=3100, num_frames=1500, H=1440, W=1920, length=230.0, spacing=0.025, size=(0.1, 0.3),
               frame_rng=True),
    # Matterport3D-region-shaped (BASELINE configs[3], dataset/matterport.py:23-24): 1280x1024 frames, depth
    # in 1/4000 m units, 2000 frames along a 300 m path, ~120k masks
    "c4": dict(num_objects=4050, num_frames=2000, H=1024, W=1280, length=300.0, spacing=0.025, size=(0.1, 0.3),
               frame_rng=True, depth_scale=4000.0),
}


def _scene(num_objects, length, spacing, size, rng):
    K = int(num_objects)
    lo_s, hi_s = size
    ext = rng.uniform(lo_s, hi_s, size=(K, 3))
    cx = np.sort(rng.uniform(0.0, length, size=K))
    cy = rng.uniform(0.2, 2.4, size=K)
    centers = np.stack([cx, cy, ext[:, 2] / 2], axis=1)
    bmin = centers - ext / 2
    bmax = centers + ext / 2
    # ---- scene points: jittered grid on the five visible faces of every box ----
    pts = []
    for o in range(K):
        for ax in range(3):
            for side in (0, 1):
                if ax == 2 and side == 0:
                    continue  # bottom face rests on the floor
                a1, a2 = [a for a in range(3) if a != ax]
                n1 = max(1, int(round(ext[o, a1] / spacing)))
                n2 = max(1, int(round(ext[o, a2] / spacing)))
                g1 = (np.arange(n1) + 0.5) / n1
                g2 = (np.arange(n2) + 0.5) / n2
                u, v = np.meshgrid(g1, g2, indexing="ij")
                f = np.zeros((u.size, 3))
                f[:, a1] = bmin[o, a1] + u.ravel() * ext[o, a1]
                f[:, a2] = bmin[o, a2] + v.ravel() * ext[o, a2]
                f[:, ax] = bmax[o, ax] if side else bmin[o, ax]
                f[:, [a1, a2]] += rng.uniform(-0.2, 0.2, size=(len(f), 2)) * spacing
                pts.append(f)
    scene = np.concatenate(pts, axis=0)
    # mesh-vertex-like order: sorted along the trajectory axis in coarse slabs
    order = np.lexsort((scene[:, 1], np.floor(scene[:, 0] / 0.25)))
    return scene[order], cx, bmin, bmax


def _cameras(F, H, W, length, yaw):
    fx = fy = 577.87 * W / 640.0
    ccx, ccy = (W - 1) / 2.0, (H - 1) / 2.0
    intr = np.tile(np.array([fx, fy, ccx, ccy]), (F, 1))
    poses = np.zeros((F, 4, 4))
    tilt = np.deg2rad(18.0)
    for f in range(F):
        psi = yaw * np.sin(0.7 * f)
        fwd = np.array([np.sin(psi) * np.cos(tilt), np.cos(psi) * np.cos(tilt), -np.sin(tilt)])
        right = np.array([np.cos(psi), -np.sin(psi), 0.0])
        down = np.cross(fwd, right)
        poses[f, :3, 0], poses[f, :3, 1], poses[f, :3, 2] = right, down, fwd
        poses[f, :3, 3] = [length * (f + 0.5) / F, -2.0, 1.3]
        poses[f, 3, 3] = 1.0
    return intr, poses


def make_frames(num_objects, num_frames, H, W, length, spacing, size, seed=0, p_split=0.06, p_merge=0.04,
                device="cpu", yaw=0.12, frame_rng=False, frames=None, out="numpy", depth_scale=1000.0):
    """Render the scene.  frames: the frame indices to render (default all; the scene points,
    intrinsics and poses always cover every frame).  frame_rng: the split / merge noise of frame f
    is drawn from its own generator (seed, f), so that any frame slice renders the same frames as
    the whole scene (the frame-sharded bench renders only each rank's slice).  out="torch": depth
    and seg stay on ``device`` as torch tensors (no host copy; the C3 frames are 21 GB)."""
    import torch

    rng = np.random.default_rng(seed)
    K = int(num_objects)
    scene, cx, bmin, bmax = _scene(num_objects, length, spacing, size, rng)
    F = int(num_frames)
    intr, poses = _cameras(F, H, W, length, yaw)
    fx, fy, ccx, ccy = intr[0]
    sel = list(range(F)) if frames is None else list(frames)

    dev = torch.device(device)
    tb0 = torch.tensor(bmin, dtype=torch.float64, device=dev)
    tb1 = torch.tensor(bmax, dtype=torch.float64, device=dev)
    u = torch.arange(W, dtype=torch.float64, device=dev)
    v = torch.arange(H, dtype=torch.float64, device=dev)
    vv, uu = torch.meshgrid(v, u, indexing="ij")
    dirs_cam = torch.stack([(uu - ccx) / fx, (vv - ccy) / fy, torch.ones_like(uu)], dim=-1).reshape(-1, 3)
    ucol = torch.arange(W, device=dev)[None, :]
    if out == "torch":
        depth = torch.zeros((len(sel), H, W), dtype=torch.float32, device=dev)
        seg = torch.zeros((len(sel), H, W), dtype=torch.uint8, device=dev)
    else:
        depth = np.zeros((len(sel), H, W), np.float32)
        seg = np.zeros((len(sel), H, W), np.uint8)
    chunk = 32 if H * W <= 400_000 else 8
    for i, f in enumerate(sel):
        R = torch.tensor(poses[f, :3, :3], dtype=torch.float64, device=dev)
        c = torch.tensor(poses[f, :3, 3], dtype=torch.float64, device=dev)
        d = dirs_cam @ R.T                       # world direction per unit camera depth
        near = np.nonzero(np.abs(cx - poses[f, 0, 3]) < 4.5)[0]
        best_t = torch.full((H * W,), float("inf"), dtype=torch.float64, device=dev)
        best_o = torch.full((H * W,), -1, dtype=torch.int64, device=dev)
        # floor (z = 0) and back wall (y = 3.2): depth without a mask
        with torch.no_grad():
            tf = torch.where(d[:, 2] < -1e-9, -c[2] / d[:, 2], torch.full_like(best_t, float("inf")))
            tw = torch.where(d[:, 1] > 1e-9, (3.2 - c[1]) / d[:, 1], torch.full_like(best_t, float("inf")))
            bg = torch.minimum(tf, tw)
            inv = 1.0 / torch.where(d.abs() < 1e-12, torch.full_like(d, 1e-12), d)
            for k0 in range(0, len(near), chunk):
                idx = torch.as_tensor(near[k0:k0 + chunk], device=dev)
                t0 = (tb0[idx][None] - c) * inv[:, None]     # [R, B, 3]
                t1 = (tb1[idx][None] - c) * inv[:, None]
                tn = torch.minimum(t0, t1).amax(-1)
                tx = torch.maximum(t0, t1).amin(-1)
                hit = (tn <= tx) & (tn > 0.05)
                tn = torch.where(hit, tn, torch.full_like(tn, float("inf")))
                tmin, arg = tn.min(-1)
                better = tmin < best_t
                best_t = torch.where(better, tmin, best_t)
                best_o = torch.where(better, idx[arg], best_o)
            use_obj = best_t < bg
            t = torch.where(use_obj, best_t, bg).reshape(H, W)
            obj = torch.where(use_obj, best_o, torch.full_like(best_o, -1)).reshape(H, W)
            # depth quantised like the uint16 PNGs (round half to even, as numpy), decoded as the datasets
            # do: float32(u16 / depth_scale) in float64 (for 1000 the same bits as a float32 division)
            dq = torch.where(torch.isfinite(t) & (t < 60.0), torch.round(t * depth_scale), torch.zeros_like(t))
            dq = torch.where(dq <= 65535.0, dq, torch.zeros_like(dq))
            dz = (dq / float(depth_scale)).to(torch.float32)
            # per-frame instance ids: visible objects in object order, with split / merge noise
            vis = torch.unique(obj[obj >= 0]).cpu().numpy()
            r = np.random.default_rng([seed, f]) if frame_rng else rng
            lab = np.zeros(K + 1, np.int64)
            nxt, j = 1, 0
            split_of = {}
            while j < len(vis) and nxt < 255:
                o = vis[j]
                lab[o + 1] = nxt
                if r.random() < p_merge and j + 1 < len(vis):
                    lab[vis[j + 1] + 1] = nxt
                    j += 1
                elif r.random() < p_split and nxt + 1 < 255:
                    split_of[o] = nxt + 1
                    nxt += 1
                nxt += 1
                j += 1
            s_ = torch.as_tensor(lab, device=dev)[obj + 1]
            for o, second in split_of.items():
                m = obj == int(o)
                cols = torch.nonzero(m.any(dim=0)).flatten()
                if len(cols) >= 2:
                    mid = int(cols[len(cols) // 2])
                    s_[m & (ucol >= mid)] = second
            s_ = s_.to(torch.uint8)
        if out == "torch":
            depth[i] = dz
            seg[i] = s_
        else:
            depth[i] = dz.cpu().numpy()
            seg[i] = s_.cpu().numpy()
    return SceneFrames(scene, depth, seg, intr[sel], poses[sel],
                       meta=dict(seed=seed, num_objects=K, length=length, spacing=spacing, frames=sel,
                                 num_frames_total=F, depth_scale=float(depth_scale)))


def make_frames_shape(name: str, seed: int = 0, device: str = "cpu", **kw) -> SceneFrames:
    params = dict(FRAME_SHAPES[name])
    params.update(kw)
    return make_frames(seed=seed, device=device, **params)
