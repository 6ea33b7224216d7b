"""Per-kernel average PMC values (and mean duration) over the rocprofv3 pass dirs of pmc_run.sh.

    python tools/pmc_by_kernel.py gpurun_out/pmc [name-substring]
"""
import collections
import csv
import glob
import re
import sys

root = sys.argv[1]
match = sys.argv[2] if len(sys.argv) > 2 else ""
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        nm = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
        if match and match not in nm:
            continue
        key = (nm, r.get("Grid_Size", r.get("Grid_Size_X", "")))
        vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for (nm, grid), cs in sorted(vals.items()):
    print(f"== {nm[:110]}  grid={grid}")
    for k, v in sorted(cs.items()):
        print(f"   {k:32s} {sum(v) / len(v):16.1f}  (n={len(v)})")
