"""Process-wide device context of the reference-API modules (graph/, utils/).

The reference keeps its tensors on the current CUDA device (``.cuda()``;
``run.py:43`` pins one GPU per process with CUDA_VISIBLE_DEVICES), so the
drop-in modules use one libmcgraph context on ``torch.cuda.current_device()``
(device 0 when torch is absent), created on first use.  There is no CPU
fallback: without the built library or a GPU the first call raises.
"""
from __future__ import annotations

import numpy as np

from . import _native

_ctx = None
_points_key = None


def context() -> _native.Context:
    global _ctx
    if _ctx is None:
        dev = 0
        try:
            import torch
            if torch.cuda.is_available():
                dev = torch.cuda.current_device()
        except ImportError:
            pass
        _ctx = _native.Context(dev)
        b = hbm_budget_from_env(dev)
        if b:
            _ctx.set_memory_budget(b)
    return _ctx


def hbm_budget_from_env(device: int = 0) -> int:
    """MASKCLUSTERING_HBM_BUDGET: the HBM bytes S1's per-batch arrays may take in the drop-in's
    context, as bytes ("60e9") or as a fraction of the device (e.g. "0.3"); unset: the library's
    default share (mc_ctx_set_memory_budget)."""
    import os
    v = os.environ.get("MASKCLUSTERING_HBM_BUDGET")
    if not v:
        return 0
    x = float(v)
    if 0 < x <= 1:
        import torch
        return int(x * torch.cuda.get_device_properties(device).total_memory)
    return int(x)


def as_numpy(x) -> np.ndarray:
    if hasattr(x, "detach"):
        return x.detach().cpu().numpy()
    return np.asarray(x)


def seg_u8(seg) -> np.ndarray:
    """A segmentation image as uint8 (mask ids <= 255: mask_predict.py:102 writes uint8 PNGs).  Ids
    outside [0, 255] would wrap and merge distinct masks, so they raise instead."""
    a = as_numpy(seg)
    if a.dtype == np.uint8:
        return a
    if a.size and (a.min() < 0 or a.max() > 255 or not np.issubdtype(a.dtype, np.integer)):
        raise ValueError(f"segmentation ids must be integers in [0, 255] (uint8 mask images); got dtype {a.dtype} "
                         f"range [{a.min()}, {a.max()}]")
    return a.astype(np.uint8)


def set_scene_points(scene_points) -> int:
    """Upload the scene points as float32 (construction.py:37) once per distinct array."""
    global _points_key
    ctx = context()
    if hasattr(scene_points, "data_ptr") and getattr(scene_points, "is_cuda", False) \
            and scene_points.dtype.__str__() == "torch.float32" and scene_points.is_contiguous():
        # always copied (device to device, cheap): a new tensor can reuse a freed tensor's block
        # with the same shape and version, so the address is no key
        ctx.set_points(device_ptr=scene_points.data_ptr(), num_points=int(scene_points.shape[0]))
        _points_key = None
        return int(scene_points.shape[0])
    pts = np.ascontiguousarray(as_numpy(scene_points), dtype=np.float32).reshape(-1, 3)
    key = ("host", pts.shape, hash(pts.tobytes()))
    if key != _points_key:
        ctx.set_points(pts)
        _points_key = key
    return len(pts)


def intrinsics_tuple(intr) -> np.ndarray:
    """fx, fy, cx, cy from an Open3D PinholeCameraIntrinsic (dataset/*.py:get_intrinsics),
    a 3x3 / 4x4 matrix, or a 4-vector."""
    if hasattr(intr, "get_focal_length"):
        fx, fy = intr.get_focal_length()
        cx, cy = intr.get_principal_point()
        return np.array([fx, fy, cx, cy], np.float64)
    if hasattr(intr, "intrinsic_matrix"):
        intr = np.asarray(intr.intrinsic_matrix)
    a = np.asarray(intr, np.float64)
    if a.shape == (4,):
        return a
    return np.array([a[0, 0], a[1, 1], a[0, 2], a[1, 2]], np.float64)


def bits_to_bool(words: np.ndarray, n: int) -> np.ndarray:
    from .pipeline import bits_to_bool as b2b
    return b2b(words, n)
