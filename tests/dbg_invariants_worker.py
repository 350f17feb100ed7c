"""Worker of tests/test_gpu_s1.py::test_diagnostics_build_invariants (run as its own process: the
library is chosen per process by MCGRAPH_LIB).

    MCGRAPH_LIB=maskclustering_amd/libmcgraph_dbg.so python tests/dbg_invariants_worker.py

With the -DMC_DBG_CHECK=1 build (built in-tree by __graft_entry__.build(), held to the spill-placement
gate like every build): every size class (MC_BP_MIN_CLASS 0..5), lists full and capped
(MC_BP_NBCAP 64 / 8), on the dense S1 inputs.  In-kernel checks recompute every list, union and k-NN
mean directly; their failure counters must stay zero, and the masks must equal the release build's
(passed in as an npz by the test).  Prints one line per case; exit 1 on any failure."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402


def main():
    from maskclustering_amd import _native
    from test_gpu_s1 import _dense_inputs, _run
    want = np.load(sys.argv[1]) if len(sys.argv) > 1 else None
    ctx = _native.Context(0)
    on, _ = ctx.debug_counters(reset=True)
    if not on:
        print("library built without in-kernel checks")
        return 1
    bad_cases = 0
    for i, inp in enumerate(_dense_inputs()):
        for min_cls in ("0", "1", "2", "3", "4", "5"):
            for nbcap in ("64", "8"):
                os.environ["MC_BP_MIN_CLASS"] = min_cls
                os.environ["MC_BP_NBCAP"] = nbcap
                got = _run(ctx, *inp)
                _, bad = ctx.debug_counters(reset=True)
                same = want is None or all(np.array_equal(want[f"in{i}_{k}"], x) for k, x in enumerate(got))
                ok = not bad.any() and same
                bad_cases += 0 if ok else 1
                print(f"input {i} class >= {min_cls} nbcap {nbcap}: failures per kind {bad.tolist()}, "
                      f"masks equal to the release build: {same}", flush=True)
    return 1 if bad_cases else 0


if __name__ == "__main__":
    sys.exit(main())
