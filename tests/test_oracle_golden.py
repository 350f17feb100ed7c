"""The CPU oracle against the reference's own outputs (golden fixtures made by
tests/golden/make_golden.py from /root/reference).  Pins the oracle before it
is trusted as the checker of the HIP path."""
import numpy as np
import pytest

import os

from conftest import CASES, GOLDEN, load_case
from golden_compare import assert_matches, case_inputs
from oracle import oracle


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_reference(name):
    z = load_case(name)
    got = oracle.run(**case_inputs(z))
    assert_matches(got, z)


def test_oracle_thresholds_unit_cases():
    z = np.load(os.path.join(GOLDEN, "unit_cases.npz"))
    for i in range(int(z["thr_cases"])):
        F = int(z[f"thr_F_{i}"])
        vf = np.unpackbits(z[f"thr_vf_{i}"], axis=1)[:, :F]
        hist = oracle.observer_hist(vf)
        thr, isint = oracle.thresholds_from_hist(hist)
        if int(z[f"thr_err_{i}"]):
            assert thr is None
            continue
        np.testing.assert_array_equal(thr.view(np.uint32), z[f"thr_val_{i}"].view(np.uint32), err_msg=f"case {i}")
        np.testing.assert_array_equal(isint, z[f"thr_isint_{i}"])


def test_oracle_percentile_matches_numpy_random():
    """np.percentile (numpy 2.x, float32 input) on random count multisets."""
    rng = np.random.default_rng(5)
    for _ in range(400):
        F = int(rng.integers(1, 60))
        n = int(rng.integers(1, 3000))
        x = rng.integers(1, F + 1, size=n).astype(np.float32)
        hist = np.bincount(x.astype(np.int64), minlength=F + 1).astype(np.uint64)
        thr, isint = oracle.thresholds_from_hist(hist)
        want = []
        for p in range(95, -5, -5):
            t = np.percentile(x, p)
            if t <= 1:
                if p < 50:
                    break
                t = 1
            want.append(t)
        assert len(want) == len(thr)
        for a, b in zip(thr, want):
            assert np.float32(a).view(np.uint32) == np.float32(b).view(np.uint32)


def test_oracle_edge_rule_unit_cases():
    z = np.load(os.path.join(GOLDEN, "unit_cases.npz"))
    vf, cm = z["ug_vf"].astype(np.uint8), z["ug_cm"].astype(np.uint8)
    N = len(vf)
    for ct_name, ct in (("0p9", 0.9), ("1", 1), ("0p8", 0.8)):
        for thr_name, thr in (("1", 1.0), ("2p5", 2.5), ("10", 10.0)):
            parts, sizes, final, _, _ = oracle.cluster(vf, cm, np.array([thr], np.float32), ct)
            A = np.unpackbits(z[f"ug_A_{ct_name}_{thr_name}"], axis=1)[:, :N].astype(bool)
            # components of the reference adjacency, min-member order
            lab = -np.ones(N, int); k = 0
            for s in range(N):
                if lab[s] >= 0: continue
                stack = [s]; lab[s] = k
                while stack:
                    u = stack.pop()
                    for v in np.nonzero(A[u])[0]:
                        if lab[v] < 0: lab[v] = k; stack.append(v)
                k += 1
            np.testing.assert_array_equal(parts[0], lab)


@pytest.mark.parametrize("name", CASES)
def test_sparse_oracle_matches_reference(name):
    """oracle/graph_sparse.c (the checker at C3/C4 sizes) against the reference's own outputs:
    every stage except the dense point-in-mask entries it never builds."""
    z = load_case(name)
    got = oracle.run_sparse(**case_inputs(z))
    got["pfm_bits"] = z["pfm_bits"]  # the sparse oracle keeps no dense point-frame matrix
    assert_matches(got, z, stages=("s3", "s5", "thr", "parts", "obj"))
    for k in ("gl_col", "gl_label", "boundary"):
        np.testing.assert_array_equal(np.asarray(got[k]), z[k], err_msg=k)


@pytest.mark.parametrize("shape,seed", [("c1", 1), ("c1", 2)])
def test_sparse_oracle_matches_dense_oracle(shape, seed):
    from maskclustering_amd.synthetic import make_shape
    s = make_shape(shape, seed=seed)
    kw = dict(mask_visible_threshold=0.3, undersegment_filter_threshold=0.3, view_consensus_threshold=0.9,
              contained_threshold=0.8)
    a = oracle.run(s.num_points, s.num_frames, s.mask_col, s.mask_label, s.mask_off, s.mask_pts, **kw)
    b = oracle.run_sparse(s.num_points, s.num_frames, s.mask_col, s.mask_label, s.mask_off, s.mask_pts, **kw)
    for k in a:
        if k.startswith("pim_") or k == "pfm_bits":
            continue
        np.testing.assert_array_equal(np.asarray(b[k]), np.asarray(a[k]), err_msg=k)
