"""Trajectory-shaped synthetic scenes for the view-consensus graph path.

This is the input generator of SURVEY.md Appendix C.  It produces exactly what
the reference's graph stage consumes from back-projection: for every frame, the
per-mask sets of scene-point ids (``mask_info`` of
``utils/mask_backprojection.py:148`` / ``frame_backprojection`` :154-156), with
mask ids 1..k in ascending order per frame (``mask_predict.py:102`` numbering,
``utils/mask_backprojection.py:77-78`` sort).

The generator is deterministic for a given seed (``numpy.random.default_rng``)
and is used by ``bench.py`` (GPU box), by the tests and by the golden-fixture
script.  It is input plumbing, not an oracle.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np


@dataclass
class SceneMasks:
    """Flat per-frame mask lists (the G-variant input of SURVEY.md §8(d)).

    Masks are in the reference's global order: frames ascending, then mask ids
    ascending (``graph/construction.py:46,55,60``).

    * ``mask_col[g]``   frame column (index into the frame list) of mask g
    * ``mask_label[g]`` the mask id inside its frame (1..255 for CropFormer PNGs)
    * ``mask_off``      CSR offsets, length M+1 (int64)
    * ``mask_pts``      scene-point ids of every mask, each segment unique
    """

    num_points: int
    num_frames: int
    mask_col: np.ndarray
    mask_label: np.ndarray
    mask_off: np.ndarray
    mask_pts: np.ndarray
    meta: dict = field(default_factory=dict)

    @property
    def num_masks(self) -> int:
        return int(self.mask_col.shape[0])

    def mask_points(self, g: int) -> np.ndarray:
        return self.mask_pts[self.mask_off[g]:self.mask_off[g + 1]]

    def per_frame_dicts(self, frame_ids=None):
        """``{frame_id: {np.uint8(id): set(point ids)}}`` — the reference's
        ``mask_dict`` shape (``utils/mask_backprojection.py:131,148``)."""
        if frame_ids is None:
            frame_ids = list(range(self.num_frames))
        out = {fid: {} for fid in frame_ids}
        for g in range(self.num_masks):
            fid = frame_ids[int(self.mask_col[g])]
            out[fid][np.uint8(self.mask_label[g]) if self.mask_label[g] < 256 else int(self.mask_label[g])] = \
                set(self.mask_points(g).tolist())
        return out

    @staticmethod
    def from_frame_lists(num_points: int, frames: list) -> "SceneMasks":
        """Build from ``frames[c] = [(label, np.ndarray points), ...]``."""
        cols, labels, lens, chunks = [], [], [], []
        for c, masks in enumerate(frames):
            for label, pts in masks:
                pts = np.asarray(pts, dtype=np.int32)
                cols.append(c)
                labels.append(int(label))
                lens.append(len(pts))
                chunks.append(pts)
        off = np.zeros(len(lens) + 1, dtype=np.int64)
        if lens:
            np.cumsum(lens, out=off[1:])
        pts = np.concatenate(chunks).astype(np.int32) if chunks else np.zeros(0, np.int32)
        return SceneMasks(num_points, len(frames), np.asarray(cols, np.int32),
                          np.asarray(labels, np.int32), off, pts)


# Shapes of SURVEY.md §8(d) (C1 is the synthetic stand-in for the demo scene).
SHAPES = {
    "few": dict(num_points=3_000, num_frames=6, num_objects=10, win=0.45),   # fewer frames than ranks (tests)
    "tiny": dict(num_points=2_000, num_frames=24, num_objects=24, win=0.12),
    "c1": dict(num_points=20_000, num_frames=100, num_objects=240, win=0.05),
    "c2": dict(num_points=240_000, num_frames=250, num_objects=600, win=0.05),
    # 2xC2 (SURVEY.md §8(d)(i)'s third point of the reference's T(M) fit): twice the frames, points
    # and objects at the same masks per frame, so M doubles
    "c2x2": dict(num_points=480_000, num_frames=500, num_objects=1200, win=0.025),
    "c3": dict(num_points=1_000_000, num_frames=1500, num_objects=2000, win=0.0133),
    "c4": dict(num_points=1_500_000, num_frames=2000, num_objects=3000, win=0.01),
}


def make_scene(num_points: int, num_frames: int, num_objects: int, win: float,
               seed: int = 0, p_split: float = 0.08, p_merge: float = 0.05,
               p_steal: float = 0.02, vis_lo: float = 0.3) -> SceneMasks:
    """Generate one scene.

    K objects are contiguous point ranges; the camera of frame f sits at f/F on
    a line and sees objects whose position is within ``win``.  Each seen object
    yields a mask of a random visible fraction of its points; masks are merged
    with the next seen object, split in halves, or steal 5 points of another
    seen object (the latter creates boundary points) with the given odds.
    Masks are shuffled and numbered 1..k in each frame.
    """
    rng = np.random.default_rng(seed)
    P, F, K = int(num_points), int(num_frames), int(num_objects)
    cuts = np.sort(rng.choice(np.arange(1, P), size=K - 1, replace=False))
    starts = np.concatenate([[0], cuts]).astype(np.int64)
    ends = np.concatenate([cuts, [P]]).astype(np.int64)
    pos = (np.arange(K) + rng.random(K)) / K

    frames = []
    for f in range(F):
        cam = f / F
        seen = np.nonzero(np.abs(pos - cam) < win)[0]
        masks = []

        def visible(o, frac):
            n = int(ends[o] - starts[o])
            keep = rng.random(n) < frac
            return (starts[o] + np.nonzero(keep)[0]).astype(np.int32)

        i = 0
        while i < len(seen):
            o = seen[i]
            pts = visible(o, rng.uniform(vis_lo, 1.0))
            if rng.random() < p_merge and i + 1 < len(seen):
                pts = np.union1d(pts, visible(seen[i + 1], 0.8)).astype(np.int32)
                i += 2
            else:
                i += 1
            parts = [pts]
            if rng.random() < p_split and len(pts) >= 2:
                h = len(pts) // 2
                parts = [pts[:h], pts[h:]]
            out_parts = []
            for part in parts:
                if rng.random() < p_steal and len(seen) > 1:
                    other = seen[rng.integers(len(seen))]
                    if other != o:
                        n = int(ends[other] - starts[other])
                        take = starts[other] + rng.choice(n, size=min(5, n), replace=False)
                        part = np.union1d(part, take.astype(np.int32)).astype(np.int32)
                if len(part):
                    out_parts.append(part)
            masks.extend(out_parts)
        order = rng.permutation(len(masks))
        frames.append([(k + 1, masks[j]) for k, j in enumerate(order)])
        # ids ascending == list order (k + 1), as the reference's sorted ids

    scene = SceneMasks.from_frame_lists(P, frames)
    scene.meta = dict(seed=seed, num_objects=K, win=win, p_split=p_split,
                      p_merge=p_merge, p_steal=p_steal)
    return scene


def make_shape(name: str, seed: int = 0, **kw) -> SceneMasks:
    params = dict(SHAPES[name])
    params.update(kw)
    return make_scene(seed=seed, **params)
