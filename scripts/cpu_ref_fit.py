"""Fit of the reference's own S2-S6 CPU time against the mask count, T(M) = a * M^b, from the
scenes scripts/cpu_ratio.py timed in the build container (C1, C2, 2xC2: profiles/cpu_ratio_*.json;
SURVEY.md §8(d)(i)), and its EXTRAPOLATION to the shapes the reference cannot run (C3, C4: dense
float32 M x M matrices, graph/construction.py:84,161, graph/iterative_clustering.py:18-21, beyond the
container's 62 GB).  Writes profiles/cpu_ref_fit.json, which bench.py quotes in
cpu_baseline.reference_context, labelled extrapolated.

    python scripts/cpu_ref_fit.py
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

# M of the shapes the fit is extrapolated to (the bench's scenes: C3 from BENCH lines, C4 likewise)
TARGETS = {"c3": 81095, "c4": 123000}


def main():
    pts = []
    for shape in ("c1", "c2", "c2x2"):
        p = os.path.join(REPO, "profiles", f"cpu_ratio_{shape}.json")
        r = json.load(open(p))
        pts.append((shape, r["M"], r["reference_s"], r["port_s"], r["host_cores"]))
    M = np.array([p[1] for p in pts], np.float64)
    T = np.array([p[2] for p in pts], np.float64)
    b, ln_a = np.polyfit(np.log(M), np.log(T), 1)
    a = float(np.exp(ln_a))
    resid = [round(float(t / (a * m ** b)), 4) for m, t in zip(M, T)]
    out = {
        "model": "T_ref(M) = a * M^b seconds, least squares in log space over the measured scenes",
        "a": a, "b": round(float(b), 4),
        "points": [{"shape": s, "M": int(m), "reference_s": t, "port_s": ps, "host_cores": hc}
                   for s, m, t, ps, hc in pts],
        "measured_over_fit": resid,
        "extrapolated_reference_s": {k: round(a * m ** b, 1) for k, m in TARGETS.items()},
        "extrapolated_M": TARGETS,
        "note": "the reference's own graph/construction.py + graph/iterative_clustering.py (S2-S6; S1 needs Open3D "
                "and pytorch3d, absent), imported unmodified (SURVEY App. B) on the 8-core build container; C3 / C4 "
                "values are EXTRAPOLATED from the fit (the reference cannot run them: dense M x M float32 matrices)",
    }
    path = os.path.join(REPO, "profiles", "cpu_ref_fit.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
