"""Sparse k6_pairs vs dense int8 MFMA for the S6 pair counts (north_star:
"sparse vs int8 MFMA chosen by measurement").

The reference forms every level's counts densely (graph/iterative_clustering.py:20-21):
supporters S = C·Cᵀ over the N_t × M contained matrix and observers O = VF·VFᵀ over N_t × F.
The dense side here is the int8 GEMM of hipBLASLt (torch._int_mm: i8 × i8 -> i32 on the matrix
cores), i.e. the best case a dense MFMA kernel of our own could reach, WITHOUT the edge-rule
epilogue, the bit unpacking or the union-find, so it is a lower bound on a dense S6.  Levels up
to --direct nodes are timed whole; larger ones as a (direct × direct) output block over the full K
and scaled by (N_t / direct)^2 (the output-area scaling of a large GEMM at fixed K).

    python scripts/s6_dense_vs_sparse.py [shape] [direct]
Run under rocprofv3 --kernel-trace --stats to get the per-launch k6_pairs durations (one per
level, in order) of the last scene step.
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from maskclustering_amd.pipeline import GraphRun  # noqa: E402
from maskclustering_amd.synthetic import make_shape  # noqa: E402

CFG = dict(mask_visible_threshold=0.3, undersegment_filter_threshold=0.3, view_consensus_threshold=0.9,
           contained_threshold=0.8)
PEAK_I8_TOPS = 5000.0  # dense int8 MFMA peak, MI355X_MICROARCH.md (no sparsity)


def pad(x, m):
    return (x + m - 1) // m * m


def time_int_mm(n, k, reps=5):
    a = torch.randint(0, 2, (n, k), dtype=torch.int8, device="cuda")
    b = torch.randint(0, 2, (k, n), dtype=torch.int8, device="cuda")
    torch._int_mm(a, b)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        torch._int_mm(a, b)
    e1.record()
    torch.cuda.synchronize()
    del a, b
    return e0.elapsed_time(e1) / reps


def main():
    shape = sys.argv[1] if len(sys.argv) > 1 else "c4"
    direct = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    t0 = time.perf_counter()
    scene = make_shape(shape, seed=0)
    print(f"{shape}: generated in {time.perf_counter() - t0:.1f} s", file=sys.stderr)
    run = GraphRun(0)
    run.set_scene(scene)
    for _ in range(2):
        run.step(**CFG)
    torch.cuda.synchronize()
    ctx = run.ctx
    ctx.reset_kernel_times()
    ctx.set_timing(True)
    run.step(**CFG)
    ctx.set_timing(False)
    torch.cuda.synchronize()
    gi, ci = ctx.graph_info(), ctx.cluster_info()
    T = ci.num_iterations
    sizes = [int(x) for x in ctx.level_sizes(T)[:T]]
    M, F = gi.num_masks, gi.num_frames
    sparse_ms = {g: round(ctx.kernel_time(g)[0], 4) for g in ("s6_columns", "s6_pairs", "s6_components", "s6_merge")}
    levels = []
    for t, n in enumerate(sizes):
        np_ = pad(max(n, 32), 64)
        row = {"t": t, "N": n}
        for name, k in (("supporters", pad(M, 64)), ("observers", pad(F, 64))):
            m = min(np_, direct)
            ms = time_int_mm(m, k)
            scale = (np_ / m) ** 2
            ops = 2.0 * m * m * k
            row[name] = {"K": k, "timed_block": m, "block_ms": round(ms, 4), "scaled_ms": round(ms * scale, 4),
                         "block_tops": round(ops / (ms * 1e-3) / 1e12, 1),
                         "mfma_frac": round(ops / (ms * 1e-3) / 1e12 / PEAK_I8_TOPS, 3)}
        row["dense_ms"] = round(row["supporters"]["scaled_ms"] + row["observers"]["scaled_ms"], 4)
        levels.append(row)
        print(json.dumps(row), file=sys.stderr, flush=True)
    out = {"shape": shape, "M": M, "F": F, "levels": T, "sizes": sizes, "sparse_s6_ms": sparse_ms,
           "sparse_s6_total_ms": round(sum(sparse_ms.values()), 4),
           "dense_gemm_total_ms": round(sum(r["dense_ms"] for r in levels), 3),
           "dense_gemm_level1_ms": levels[1]["dense_ms"] if T > 1 else None,
           "note": "dense = hipBLASLt int8 GEMMs only (torch._int_mm), no epilogue: a lower bound on a dense S6",
           "per_level": levels}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
