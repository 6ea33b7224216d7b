"""Average every PMC counter per kernel (name filter) over the pmc_run.sh passes, plus derived issue figures.

    python tools/pmc_dump.py gpurun_out/<run> <substring> [<substring> ...]
"""
import collections
import csv
import glob
import re
import sys

root, pats = sys.argv[1], sys.argv[2:]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        nm = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
        if pats and not any(p in nm for p in pats):
            continue
        vals[(nm, r.get("Grid_Size", ""))][r["Counter_Name"]].append(float(r["Counter_Value"]))
for (nm, grid), cs in sorted(vals.items()):
    a = {k: sum(v) / len(v) for k, v in cs.items()}
    print(f"== {nm} grid {grid}")
    for k in sorted(a):
        print(f"   {k:28s} {a[k]:16.0f}")
    wc = a.get("SQ_WAVE_CYCLES")
    if wc:
        print("   wave-cycle split: active %.2f  issue-stall %.2f  parked(waitcnt/barrier) %.2f  lds-issue-stall %.2f"
              % (a.get("SQ_ACTIVE_INST_ANY", 0) / wc, a.get("SQ_WAIT_INST_ANY", 0) / wc, a.get("SQ_WAIT_ANY", 0) / wc,
                 a.get("SQ_WAIT_INST_LDS", 0) / wc))
    if "GRBM_GUI_ACTIVE" in a:
        cyc = a["GRBM_GUI_ACTIVE"] / 8
        if "SQ_VALU_MFMA_BUSY_CYCLES" in a:
            print("   MFMA busy %.3f   VALU busy (INSTS_VALU x 2 cyc) %.3f   (per SIMD, over %.0f cycles)"
                  % (a["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / cyc, a.get("SQ_INSTS_VALU", 0) * 2 / 1024 / cyc, cyc))
