"""Per-kernel memory-side traffic from the L2's request-size counters (rocprofv3 --pmc passes, one CSV
per pass), without the blanket FETCH_SIZE doubling (verdict r4 item 7).

gfx950's FETCH_SIZE is derived as (TCC_BUBBLE*128 + (RDREQ - BUBBLE - RDREQ_32B)*64 + RDREQ_32B*32) and
reads half of the bytes of a wide streaming read (MI355X_MICROARCH.md §HBM: 128-byte requests tallied at
64 B).  The size-split counters say what each kernel's requests were:
  read bytes  = 32*RDREQ_32B + 64*RDREQ_64B + 128*RDREQ_128B        (every request by its size)
  read bytes' = 32*RDREQ_DRAM_32B                                    (DRAM-bound requests in 32-B units)
  write bytes = 32*(WRREQ - WRREQ_64B) + 64*WRREQ_64B                (WRITE_SIZE's own definition)
  write bytes'= 32*WRREQ_WRITE_DRAM_32B
The two read figures cross-check each other; the reported traffic is the size-split one, and the share
of 32-B requests (partial lines) is reported beside it.  Infinity-Cache hits are counted as memory-side
traffic by these counters (the guide), so this is L2-miss traffic, an upper bound on HBM bytes.

    python scripts/pmc_sizes.py <dir with sizes*.csv> <out.json> [kernel-regex]
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def load(d):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))  # kernel -> counter -> per dispatch
    for path in sorted(glob.glob(os.path.join(d, "sizes*.csv"))):
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"].replace("void ", "").split("(")[0]
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return vals


def main():
    d, out = sys.argv[1], sys.argv[2]
    rx = re.compile(sys.argv[3]) if len(sys.argv) > 3 else None
    vals = load(d)
    res = {"source": d, "units": "bytes per dispatch (average over dispatches)", "kernels": {}}
    for k, cs in sorted(vals.items()):
        if rx and not rx.search(k):
            continue
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        g = lambda c: avg.get(c + "_sum", avg.get(c, 0.0))  # noqa: E731
        rd = 32 * g("TCC_EA0_RDREQ_32B") + 64 * g("TCC_EA0_RDREQ_64B") + 128 * g("TCC_EA0_RDREQ_128B")
        rd_dram = 32 * g("TCC_EA0_RDREQ_DRAM_32B")
        wr = 32 * (g("TCC_EA0_WRREQ") - g("TCC_EA0_WRREQ_64B")) + 64 * g("TCC_EA0_WRREQ_64B")
        wr_dram = 32 * g("TCC_EA0_WRREQ_WRITE_DRAM_32B")
        fetch_size = (128 * g("TCC_BUBBLE") + 64 * (g("TCC_EA0_RDREQ") - g("TCC_BUBBLE") - g("TCC_EA0_RDREQ_32B"))
                      + 32 * g("TCC_EA0_RDREQ_32B"))
        nreq = g("TCC_EA0_RDREQ_32B") + g("TCC_EA0_RDREQ_64B") + g("TCC_EA0_RDREQ_128B")
        res["kernels"][k] = {
            "dispatches": max(len(v) for v in cs.values()),
            "read_bytes": rd, "read_bytes_dram32": rd_dram, "write_bytes": wr, "write_bytes_dram32": wr_dram,
            "fetch_size_formula_bytes": fetch_size,
            "read_req_share_32B": g("TCC_EA0_RDREQ_32B") / nreq if nreq else None,
            "read_req_share_128B": g("TCC_EA0_RDREQ_128B") / nreq if nreq else None,
            "write_req_share_64B": g("TCC_EA0_WRREQ_64B") / g("TCC_EA0_WRREQ") if g("TCC_EA0_WRREQ") else None,
            "counters": avg,
        }
    json.dump(res, open(out, "w"), indent=1)
    for k, v in res["kernels"].items():
        print(f"{k[:48]:48s} rd {v['read_bytes'] / 1e6:9.1f} MB (dram32 {v['read_bytes_dram32'] / 1e6:9.1f}, "
              f"FETCH_SIZE {v['fetch_size_formula_bytes'] / 1e6:9.1f}) wr {v['write_bytes'] / 1e6:9.1f} MB "
              f"(dram32 {v['write_bytes_dram32'] / 1e6:9.1f}) 32B-read share {v['read_req_share_32B']}")


if __name__ == "__main__":
    main()
