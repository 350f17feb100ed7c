"""Average per-dispatch PMC counters of the kernels matching a name fragment, from
rocprofv3 --pmc counter_collection.csv files (one per pass).

    python scripts/pmc_kernel.py <fragment> <csv> [<csv> ...]
"""
import collections
import csv
import json
import sys


def main():
    frag, paths = sys.argv[1], sys.argv[2:]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            name = r["Kernel_Name"].replace("void ", "").split("(")[0]
            if frag in name:
                acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {k: {c: round(sum(v) / len(v), 1) for c, v in sorted(cs.items())} for k, cs in acc.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
