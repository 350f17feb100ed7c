"""HIP path (through the C-ABI) against the reference's golden outputs and the
CPU oracle.  Bit-exact: every quantity on this path is integer/index work."""
import os

import numpy as np
import pytest

from conftest import CASES, GOLDEN, load_case
from golden_compare import assert_matches, case_inputs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def run():
    from maskclustering_amd.pipeline import GraphRun
    return GraphRun(0)


def _run_case(run, inp):
    run.set_masks(inp["num_points"], inp["num_frames"], inp["mask_col"], inp["mask_label"], inp["mask_off"],
                  inp["mask_pts"])
    run.step(inp["mask_visible_threshold"], inp["undersegment_filter_threshold"],
             inp["view_consensus_threshold"], inp["contained_threshold"])
    return run.canonical()


@pytest.mark.parametrize("name", CASES)
def test_graph_path_matches_reference(run, name):
    z = load_case(name)
    got = _run_case(run, case_inputs(z))
    assert_matches(got, z)
    np.testing.assert_array_equal(got["edge_counts"], z["edge_counts"], err_msg="edges per iteration")


def test_observer_thresholds_unit_cases(run):
    from maskclustering_amd.pipeline import bool_to_bits
    from maskclustering_amd._native import McError, MC_ERR_EMPTY_OBSERVERS
    z = np.load(os.path.join(GOLDEN, "unit_cases.npz"))
    for i in range(int(z["thr_cases"])):
        F = int(z[f"thr_F_{i}"])
        vf = np.unpackbits(z[f"thr_vf_{i}"], axis=1)[:, :F].astype(bool)
        if int(z[f"thr_err_{i}"]):
            with pytest.raises(McError) as e:
                run.ctx.observer_thresholds(bool_to_bits(vf), F)
            assert e.value.code == MC_ERR_EMPTY_OBSERVERS
            continue
        thr, isint = run.ctx.observer_thresholds(bool_to_bits(vf), F)
        np.testing.assert_array_equal(thr.view(np.uint32), z[f"thr_val_{i}"].view(np.uint32), err_msg=f"case {i}")
        np.testing.assert_array_equal(isint, z[f"thr_isint_{i}"])


def _components(A):
    N = len(A)
    lab = -np.ones(N, int)
    k = 0
    for s in range(N):
        if lab[s] >= 0:
            continue
        stack = [s]
        lab[s] = k
        while stack:
            u = stack.pop()
            for v in np.nonzero(A[u])[0]:
                if lab[v] < 0:
                    lab[v] = k
                    stack.append(v)
        k += 1
    return lab


def _set_nodes_dense(run, vf, cm, pts=None):
    from maskclustering_amd.pipeline import bool_to_bits
    N, F = vf.shape
    M = cm.shape[1]
    r, c = np.nonzero(cm)
    c_off = np.zeros(N + 1, np.int64)
    c_off[1:] = np.cumsum(np.bincount(r, minlength=N))
    if pts is None:
        pts = [np.array([i], np.int32) for i in range(N)]
    pt_off = np.zeros(N + 1, np.int64)
    pt_off[1:] = np.cumsum([len(p) for p in pts])
    P = int(max((p.max() + 1 for p in pts if len(p)), default=1))
    run.ctx.set_nodes(F, M, P, bool_to_bits(vf.astype(bool)), c_off, c.astype(np.int32), pt_off,
                      np.concatenate(pts).astype(np.int32))


def test_edge_rule_unit_cases(run):
    """Float32 rate boundaries (S = 0.9·O exactly, O = 1 with ct = 1, ...)."""
    z = np.load(os.path.join(GOLDEN, "unit_cases.npz"))
    vf, cm = z["ug_vf"] > 0, z["ug_cm"] > 0
    N = len(vf)
    for ct_name, ct in (("0p9", 0.9), ("1", 1), ("0p8", 0.8)):
        for thr_name, thr in (("1", 1.0), ("2p5", 2.5), ("10", 10.0)):
            _set_nodes_dense(run, vf, cm)
            run.cluster(ct, thresholds=np.array([thr], np.float32))
            A = np.unpackbits(z[f"ug_A_{ct_name}_{thr_name}"], axis=1)[:, :N].astype(bool)
            np.testing.assert_array_equal(run.ctx.partition(0, N), _components(A), err_msg=f"{ct_name} {thr_name}")


def _oracle_cluster_check(run, vf, cm, thr, ct):
    from oracle import oracle
    parts, sizes, final, fvf, fcm = oracle.cluster(vf.astype(np.uint8), cm.astype(np.uint8), np.asarray(thr, np.float32), ct)
    _set_nodes_dense(run, vf, cm)
    run.cluster(ct, thresholds=np.asarray(thr, np.float32))
    got = run.canonical_cluster(vf.shape[1])
    assert int(got["num_iters"]) == len(parts)
    for t in range(len(parts)):
        np.testing.assert_array_equal(got[f"part_{t}"], parts[t], err_msg=f"partition {t}")
    np.testing.assert_array_equal(run.ctx.final_labels(len(vf)), final)
    from maskclustering_amd.pipeline import bits_to_bool
    K = len(fvf)
    obj = run.ctx.objects(run.ctx.cluster_info(), vf.shape[1])
    np.testing.assert_array_equal(bits_to_bool(obj["vf_bits"], vf.shape[1]), fvf.astype(bool))
    for k in range(K):
        np.testing.assert_array_equal(obj["c_idx"][obj["c_off"][k]:obj["c_off"][k + 1]], np.nonzero(fcm[k])[0])


def test_hash_overflow_path(run):
    """A node with > 768 distinct supporter partners goes through the overflow kernel."""
    N, M, F = 1400, 1400, 40
    rng = np.random.default_rng(0)
    vf = np.zeros((N, F), bool)
    vf[:, :20] = True
    cm = np.zeros((N, M), bool)
    cm[0, :N - 1] = True              # node 0 shares a mask with every other node
    for b in range(1, N):
        cm[b, b - 1] = True
        cm[b, rng.integers(0, M)] = True
    _oracle_cluster_check(run, vf, cm, [1.0, 1.0], 0.05)


def test_dense_observer_path_ct_zero(run):
    rng = np.random.default_rng(1)
    N, F, M = 300, 50, 200
    vf = rng.random((N, F)) < 0.1
    cm = rng.random((N, M)) < 0.02
    _oracle_cluster_check(run, vf, cm, [4.0, 3.0, 2.0], 0.0)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_random_nodes_vs_oracle(run, seed):
    rng = np.random.default_rng(10 + seed)
    N, F, M = 500, 64 + 7 * seed, 400
    vf = rng.random((N, F)) < 0.15
    cm = (rng.random((N, M)) < 0.03) & np.repeat(rng.random((N, 1)) < 0.9, M, axis=1)
    _oracle_cluster_check(run, vf, cm, [5.0, 3.5, 2.0, 1.0], [0.9, 0.5, 1.0][seed])


@pytest.mark.parametrize("shape,seed,cfg", [("c2", 0, (0.3, 0.3, 0.9, 0.8)), ("c1", 3, (0.4, 0.2, 1, 0.9)),
                                            ("c1", 4, (0.2, 0.1, 0.9, 0.8))])
def test_synthetic_scene_vs_oracle(run, shape, seed, cfg):
    from maskclustering_amd.synthetic import make_shape
    from oracle import oracle
    s = make_shape(shape, seed=seed)
    mvt, ust, ct, cont = cfg
    want = oracle.run(s.num_points, s.num_frames, s.mask_col, s.mask_label, s.mask_off, s.mask_pts, mvt, ust, ct, cont)
    inp = dict(num_points=s.num_points, num_frames=s.num_frames, mask_col=s.mask_col, mask_label=s.mask_label,
               mask_off=s.mask_off, mask_pts=s.mask_pts, mask_visible_threshold=mvt,
               undersegment_filter_threshold=ust, view_consensus_threshold=ct, contained_threshold=cont)
    got = _run_case(run, inp)
    assert_matches(got, want)


def test_repeat_is_deterministic(run):
    from maskclustering_amd.synthetic import make_shape
    s = make_shape("c1", seed=5)
    inp = dict(num_points=s.num_points, num_frames=s.num_frames, mask_col=s.mask_col, mask_label=s.mask_label,
               mask_off=s.mask_off, mask_pts=s.mask_pts, mask_visible_threshold=0.3,
               undersegment_filter_threshold=0.3, view_consensus_threshold=0.9, contained_threshold=0.8)
    a = _run_case(run, inp)
    run.step(0.3, 0.3, 0.9, 0.8)
    b = run.canonical()
    for k in a:
        np.testing.assert_array_equal(np.asarray(a[k]), np.asarray(b[k]), err_msg=k)


def test_s3_pair_table_overflow(run):
    """S3 masks meeting more (frame, mask) pairs than the LDS hash table holds (512 for
    wave masks, 2048 for workgroup masks) take the dense-counter path; results must not
    change.  Frames 0..199 cut the points into 12 random masks each (2400 pairs per point
    set); frame 200 adds a 1000-point mask (wave kernel), frame 201 a 4000-point mask
    (workgroup kernel), frame 202 small masks that stay in the table."""
    from maskclustering_amd.synthetic import SceneMasks
    from oracle import oracle
    rng = np.random.default_rng(7)
    P = 4000
    frames = []
    for _ in range(200):
        part = rng.integers(0, 12, P)
        frames.append([(k + 1, np.nonzero(part == k)[0]) for k in range(12)])
    frames.append([(1, np.arange(1000)), (2, np.arange(1000, 1500))])
    frames.append([(3, np.arange(P))])
    frames.append([(k + 1, np.arange(3000 + 40 * k, 3040 + 40 * k)) for k in range(5)])
    s = SceneMasks.from_frame_lists(P, frames)
    for cfg in ((0.05, 0.5, 0.5, 0.1), (0.2, 0.99, 0.9, 0.15)):  # configs with visible frames
        mvt, ust, ct, cont = cfg
        want = oracle.run(s.num_points, s.num_frames, s.mask_col, s.mask_label, s.mask_off, s.mask_pts,
                          mvt, ust, ct, cont)
        inp = dict(num_points=s.num_points, num_frames=s.num_frames, mask_col=s.mask_col, mask_label=s.mask_label,
                   mask_off=s.mask_off, mask_pts=s.mask_pts, mask_visible_threshold=mvt,
                   undersegment_filter_threshold=ust, view_consensus_threshold=ct, contained_threshold=cont)
        assert_matches(_run_case(run, inp), want)
