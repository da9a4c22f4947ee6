"""Median per-dispatch value of every counter in rocprofv3 counter_collection CSVs, by kernel name.

    python tools/pmc_by_kernel.py gpurun_out/pmc_s2_a gpurun_out/pmc_s2_b ...
"""
import collections
import csv
import statistics
import sys
from pathlib import Path


def main():
    per = collections.defaultdict(lambda: collections.defaultdict(dict))  # kernel -> dispatch -> counter
    for d in sys.argv[1:]:
        for f in Path(d).glob("*counter_collection.csv"):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                per[k][(d, r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    for k, disp in per.items():
        agg = collections.defaultdict(list)
        for cs in disp.values():
            for c, v in cs.items():
                agg[c].append(v)
        print(k[:90])
        for c in sorted(agg):
            print(f"    {c:24s} {statistics.median(agg[c]):.4g}  (n={len(agg[c])})")


if __name__ == "__main__":
    main()
