"""The post-processing oracle (oracle/pp_oracle.py) against the reference's own
post_process outputs (tests/golden/pp_small.npz, made by tests/golden/make_pp_golden.py)."""
import os

import numpy as np
import pytest

from oracle import pp_oracle

GOLD = os.path.join(os.path.dirname(__file__), "golden", "pp_small.npz")


def load_case(z, c):
    mask_pts = [z["mpc_idx"][z["mpc_off"][i]:z["mpc_off"][i + 1]] for i in range(len(z["mpc_col"]))]
    mo, mi = z[c + "_node_mask_off"], z[c + "_node_mask_idx"]
    po, pi_ = z[c + "_node_pt_off"], z[c + "_node_pt_idx"]
    nodes = [(mi[mo[k]:mo[k + 1]].tolist(), z[c + "_node_vf"][k], pi_[po[k]:po[k + 1]])
             for k in range(len(mo) - 1)]
    return mask_pts, nodes


def expected(z, c):
    oo, oi = z[c + "_obj_pt_off"], z[c + "_obj_pt_idx"]
    qo, qi, qc = z[c + "_obj_mask_off"], z[c + "_obj_mask_idx"], z[c + "_obj_mask_cov"]
    pts = [oi[oo[k]:oo[k + 1]] for k in range(len(oo) - 1)]
    masks = [list(zip(qi[qo[k]:qo[k + 1]].tolist(), qc[qo[k]:qo[k + 1]].tolist())) for k in range(len(qo) - 1)]
    return pts, masks


def assert_same(got, want):
    gp, gm = got
    wp, wm = want
    assert len(gp) == len(wp)
    for k in range(len(wp)):
        np.testing.assert_array_equal(np.asarray(gp[k], np.int64), wp[k].astype(np.int64), err_msg=f"object {k} points")
        assert [m for m, _ in gm[k]] == [m for m, _ in wm[k]], f"object {k} masks"
        # coverage is a Python float in the reference: bit-exact
        assert [float(c) for _, c in gm[k]] == [c for _, c in wm[k]], f"object {k} coverage"


@pytest.mark.parametrize("case", ["a", "b"])
def test_pp_oracle_matches_reference(case):
    z = np.load(GOLD)
    mask_pts, nodes = load_case(z, case)
    got = pp_oracle.post_process_objects(z["scene"], z["pfm"], mask_pts, z["mpc_col"], nodes, float(z[case + "_thr"]))
    assert_same(got, expected(z, case))


def test_pp_oracle_dbscan_known_answers():
    # two blobs + an isolated point + a border point reached from cluster 1 first
    p = np.array([[0, 0, 0], [0.05, 0, 0], [0, 0.05, 0], [0.05, 0.05, 0],      # blob A (core)
                  [5, 5, 5],                                                     # noise
                  [1, 0, 0], [1.05, 0, 0], [1, 0.05, 0], [1.05, 0.05, 0]], float)  # blob B
    lab = pp_oracle.dbscan(p, 0.1, 4)
    assert lab.tolist() == [0, 0, 0, 0, -1, 1, 1, 1, 1]
    # order matters for numbering: B first
    lab2 = pp_oracle.dbscan(p[[5, 6, 7, 8, 0, 1, 2, 3, 4]], 0.1, 4)
    assert lab2.tolist() == [0, 0, 0, 0, 1, 1, 1, 1, -1]
