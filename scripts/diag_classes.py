"""Diagnostic: run the tiny dense S1 scene of test_denoise_size_classes_match_oracle under every
MC_BP_MIN_CLASS, REPS times each, and print every candidate-statistics element that differs from the
oracle and from the first run (slot, column, values)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from maskclustering_amd import _native  # noqa: E402
from maskclustering_amd.synthetic_frames import make_frames_shape  # noqa: E402

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 4
COLS = ["frame", "id", "npix", "nvox", "ndbscan", "nsor", "ncand", "ncovered", "nneighbors", "kept"]
fr = make_frames_shape("tiny", seed=5, H=360, W=480, num_frames=3)
ctx = _native.Context(0)
ctx.set_points(fr.scene_points.astype(np.float32))


def run():
    ctx.backproject(fr.depth, fr.seg, fr.intrinsics, fr.poses)
    return ctx.bp_candidates().copy()


os.environ.pop("MC_BP_MIN_CLASS", None)
ref = run()
# the oracle's statistics of the same frames (oracle/s1_oracle.c): which run is right
from oracle import oracle  # noqa: E402  (diagnostic: the checker)
want = oracle.s1_frames(fr.scene_points.astype(np.float32), fr.depth, fr.seg, fr.intrinsics, fr.poses)
CMP = [(1, 0), (2, 1), (3, 2), (4, 3), (5, 4), (7, 6), (8, 7), (9, 8)]


def vs_oracle(st):
    out = []
    for c, (ol, oo, op, ost) in enumerate(want):
        big = ost[ost[:, 1] >= 25]
        dev = st[st[:, 0] == c]
        if len(dev) != len(big):
            out.append(f"frame {c}: {len(dev)} candidates vs {len(big)}")
            continue
        for dc, oc in CMP:
            bad = np.nonzero(dev[:, dc] != big[:, oc])[0]
            for i in bad[:4]:
                out.append(f"frame {c} id {dev[i, 1]} {COLS[dc]} {dev[i, dc]} (oracle {big[i, oc]})")
    return out


print("default run vs oracle:", vs_oracle(ref) or "equal", flush=True)
bad = 0
for per_class in ("-",):
    for mc in ("0", "1", "2", "3", "4", "5", "6"):
        os.environ["MC_BP_MIN_CLASS"] = mc
        for r in range(REPS):
            if os.environ.get("DIAG_VERBOSE"):
                print(f"-- run per_class={per_class} min_class={mc} rep={r}", flush=True)
            got = run()
            vo = vs_oracle(got)
            if vo:
                print(f"per_class={per_class} min_class={mc} rep={r} vs oracle: " + "; ".join(vo[:6]), flush=True)
            d = np.argwhere(got != ref)
            if len(d):
                bad += 1
                print(f"per_class={per_class} min_class={mc} rep={r}: " + "; ".join(
                    f"slot {i} (frame {ref[i, 0]} id {ref[i, 1]} nvox {ref[i, 3]}) {COLS[j]} {ref[i, j]} -> {got[i, j]}"
                    for i, j in d[:8]), flush=True)
print("differing runs", bad, "of", 7 * REPS, flush=True)
