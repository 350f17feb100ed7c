"""Per-kernel-group HBM traffic per launch from two rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE, kilobytes per dispatch), corrected as
MI355X_MICROARCH.md §HBM prescribes for gfx950: FETCH_SIZE counts half of the
bytes of wide coalesced reads, so it is doubled; WRITE_SIZE is taken as is.
(Access widths other than 16 B/lane are uncalibrated; the ratio against the
algorithmic bytes is what the bench line reports.)

    python scripts/pmc_summary.py <dir with pmc_FETCH_SIZE.csv, pmc_WRITE_SIZE.csv> <out.json>
"""
import collections
import csv
import json
import os
import sys

# timed group of mc_api.hip (TimedScope names) -> (kernel-name prefixes, anchor prefixes): a group
# launch is one launch of an anchor kernel (TimedScope count), and its bytes are the total bytes of
# all the group's kernels over the anchor launches.  An anchor must launch exactly once per timed
# scope: k_bp_vox_order launches twice per batch (once in bp_voxel's scope, once in bp_denoise's,
# mc_api.hip), so bp_voxel anchors on its first LDS tier and SHARED splits vox_order between the two.
SHARED = {"mc::k_bp_vox_order": {"bp_voxel": 0.5, "bp_denoise": 0.5}}
GROUPS = {
    "s3_masks": (["mc::k_s3_masks"], ["mc::k_s3_masks<1>"]),
    "s2_point_lists": (["mc::k_s2_degree", "mc::k_s2_scatter", "mc::k_s2_points", "mc::k_scan_reduce",
                        "mc::k_scan_down"], ["mc::k_s2_degree"]),
    "s3_undo_s5": (["mc::k_s3_undo", "mc::k_s5_nodes"], ["mc::k_s5_nodes"]),
    "s4_observer_hist": (["mc::k_s4_hist", "mc::k_s4_ranges", "mc::k_s4_thresholds"], ["mc::k_s4_thresholds"]),
    "s6_columns": (["mc::k6_colcount", "mc::k6_colscatter", "mc::k6_colupdate"], ["mc::k6_colcount"]),
    "s6_pairs": (["mc::k6_pairs"], ["mc::k6_pairs"]),
    "s6_components": (["mc::k6_components", "mc::k6_compress", "mc::k6_relabel", "mc::k6_memscatter"],
                      ["mc::k6_components", "mc::k6_compress"]),
    "s6_merge": (["mc::k6_merge"], ["mc::k6_merge"]),
    "s7_points": (["mc::k7"], ["mc::k7_words", "mc::k7_count"]),
    "bp_grid": (["mc::k_grid_count", "mc::k_grid_scatter"], ["mc::k_grid_count"]),
    "bp_pixels": (["mc::k_bp_count", "mc::k_bp_frames", "mc::k_bp_slots", "mc::k_bp_compact"], ["mc::k_bp_count"]),
    "bp_voxel": (["mc::k_bp_voxel", "mc::k_bp_vox_order"], ["mc::k_bp_voxel_lds<256"]),
    "bp_denoise": (["mc::k_bp_denoise", "mc::k_bp_classify", "mc::k_bp_knn_ring", "mc::k_bp_vox_order"],
                   ["mc::k_bp_classify"]),
    "bp_query": (["mc::k_bp_query", "mc::k_bp_keepflags", "mc::k_bp_emit"], ["mc::k_bp_query", "mc::k_bp_emit"]),
}


def per_kernel(path):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        name = name.replace("void ", "")
        agg[name.split("(")[0]].append(float(r["Counter_Value"]))
    return agg


def main():
    d, out = sys.argv[1], sys.argv[2]
    fetch = per_kernel(os.path.join(d, "pmc_FETCH_SIZE.csv"))
    write = per_kernel(os.path.join(d, "pmc_WRITE_SIZE.csv"))
    res = {"source": d, "correction": "bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE halving)",
           "kernels": {}, "groups": {}}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, []), write.get(k, [])
        res["kernels"][k] = {"launches": max(len(f), len(w)),
                             "fetch_kb_avg": sum(f) / max(len(f), 1), "write_kb_avg": sum(w) / max(len(w), 1)}
    for g, (prefixes, anchors) in GROUPS.items():
        ks = [k for k in res["kernels"] if any(k.startswith(p) for p in prefixes)]
        n = sum(res["kernels"][k]["launches"] for k in res["kernels"] if any(k.startswith(p) for p in anchors))
        if not ks or not n:
            continue
        kk = res["kernels"]
        share = {k: next((w[g] for p, w in SHARED.items() if k.startswith(p) and g in w), 1.0) for k in ks}
        per_k = {k: share[k] * (2 * kk[k]["fetch_kb_avg"] + kk[k]["write_kb_avg"]) * 1024 * kk[k]["launches"] / n
                 for k in ks}
        res["groups"][g] = {"bytes_per_launch": sum(per_k.values()), "kernels": ks, "group_launches": n,
                            "bytes_per_launch_by_kernel": per_k}
    json.dump(res, open(out, "w"), indent=1)
    for g, v in res["groups"].items():
        print(f"{g:20s} {v['bytes_per_launch'] / 1e6:10.2f} MB/launch")


if __name__ == "__main__":
    main()
