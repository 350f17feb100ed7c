"""Shared comparison of a pipeline result against a golden fixture (canonical,
order-free form: SURVEY.md §8(c), App. A.7)."""
import numpy as np

STAGE_KEYS = {
    "s2": ["gl_col", "gl_label", "boundary", "pim_p", "pim_c", "pim_v", "pfm_bits"],
    "s3": ["vf_bits", "c_row", "c_col", "undersegment"],
    "s5": ["node0_g"],
    "obj": ["obj_mask_off", "obj_mask_idx", "obj_pt_off", "obj_pt_idx", "obj_vf_bits",
            "obj_c_off", "obj_c_idx", "obj_node_info", "obj_son_off", "obj_son_idx"],
}


def case_inputs(z):
    cfg = z["cfg"]
    ct = int(cfg[2]) if bool(z["cfg_ct_is_int"]) else float(cfg[2])
    return dict(num_points=int(z["in_num_points"]), num_frames=int(z["in_num_frames"]),
                mask_col=z["in_mask_col"], mask_label=z["in_mask_label"], mask_off=z["in_mask_off"],
                mask_pts=z["in_mask_pts"], mask_visible_threshold=float(cfg[0]),
                undersegment_filter_threshold=float(cfg[1]), view_consensus_threshold=ct,
                contained_threshold=float(cfg[3]))


def assert_matches(got, want, stages=("s2", "s3", "s5", "thr", "parts", "obj")):
    for st in stages:
        if st == "thr":
            np.testing.assert_array_equal(np.asarray(got["thr_value"], np.float32).view(np.uint32),
                                          want["thr_value"].view(np.uint32), err_msg="thresholds (f32 bits)")
            np.testing.assert_array_equal(np.asarray(got["thr_is_int"], bool), want["thr_is_int"],
                                          err_msg="threshold int-1 substitution")
        elif st == "parts":
            assert int(got["num_iters"]) == int(want["num_iters"])
            for t in range(int(want["num_iters"])):
                np.testing.assert_array_equal(got[f"part_{t}"], want[f"part_{t}"], err_msg=f"partition {t}")
        else:
            for k in STAGE_KEYS[st]:
                np.testing.assert_array_equal(np.asarray(got[k]), want[k], err_msg=k)
