"""Packed per-scene frames: the step before the path.

The reference reads every frame from files (dataset/scannet.py:44-73: pose txt, uint16 depth PNG
divided by ``depth_scale``, uint8 segmentation PNG resized to the depth size with
cv2.INTER_NEAREST) one frame at a time on the host.  A scene pack keeps the raw frames of one
scene in one uncompressed ``.npz`` (no pickle): depth uint16 [F, H, W] as stored in the PNGs,
segmentation uint8 [F, Hs, Ws] at its own size, intrinsics [F, 4] (fx, fy, cx, cy), poses
[F, 4, 4], frame ids, ``depth_scale``.  ``load_scene_pack`` moves the raw arrays to the device
and decodes them there in one launch (``mc_frames_decode``: the float64 division and the
nearest-neighbour resize), giving exactly the arrays ``mc_backproject`` reads.
"""
from __future__ import annotations

import numpy as np

from . import _device


def write_scene_pack(path, depth_u16, seg, intrinsics, poses, frame_ids, depth_scale):
    depth_u16 = np.asarray(depth_u16)
    if depth_u16.dtype != np.uint16:
        raise TypeError("depth must be the uint16 values of the depth PNGs")
    np.savez(path, depth=depth_u16, seg=np.asarray(seg, np.uint8), intrinsics=np.asarray(intrinsics, np.float64),
             poses=np.asarray(poses, np.float64).reshape(-1, 4, 4), frame_ids=np.asarray(frame_ids),
             depth_scale=np.float64(depth_scale))


def decode_frames(depth_u16, seg, depth_scale, device="cuda:0"):
    """Device tensors (float32 depth [F, H, W], uint8 seg [F, H, W]) from raw frames (numpy or
    device tensors): dataset/scannet.py:52-53 and :72 for every frame in one launch."""
    import torch
    dev = torch.device(device)
    d = torch.as_tensor(np.asarray(depth_u16) if not torch.is_tensor(depth_u16) else depth_u16)
    s = torch.as_tensor(np.asarray(seg) if not torch.is_tensor(seg) else seg)
    d = d.to(dev).contiguous()
    s = s.to(dev, torch.uint8).contiguous()
    F, H, W = d.shape
    Hs, Ws = s.shape[1:]
    depth_out = torch.empty((F, H, W), dtype=torch.float32, device=dev)
    seg_out = torch.empty((F, H, W), dtype=torch.uint8, device=dev)
    ctx = _device.context()
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    ctx.frames_decode(F, H, W, d.data_ptr(), float(depth_scale), (Hs, Ws), s.data_ptr(), True,
                      depth_out.data_ptr(), seg_out.data_ptr())
    return depth_out, seg_out


def load_scene_pack(path, device="cuda:0"):
    z = np.load(path)
    depth, seg = decode_frames(z["depth"], z["seg"], float(z["depth_scale"]), device)
    return dict(depth=depth, seg=seg, intrinsics=z["intrinsics"], poses=z["poses"],
                frame_ids=z["frame_ids"].tolist())
