"""Average PMC counter values per dispatch of kernels matching a substring, over rocprofv3 pass dirs.

    python tools/pmc_summary.py gpurun_out/pmc [kernel-substring]
"""
import collections
import csv
import glob
import sys

root = sys.argv[1]
match = sys.argv[2] if len(sys.argv) > 2 else "gemm"
vals = collections.defaultdict(list)
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if match not in r["Kernel_Name"]:
            continue
        vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in vals.items():
    print(f"{k:36s} {sum(v) / len(v):16.1f}  (n={len(v)})")
