"""Per-kernel issue-bound summary from the pmc_run.sh passes: VALU pipe busy (SQ_INSTS_VALU x 2 cycles per
wave64 instruction -- a SIMD retires 32 f32 FMA lanes per cycle, tools/valu_rate.hip -- over 1024 SIMDs, against
GRBM_GUI_ACTIVE / 8 XCDs), the wave-cycle split (active /
issue-stalled / parked on s_waitcnt or a barrier; SQ_* quad-cycle units cancel), and FETCH / WRITE bytes.

    python tools/pmc_valu.py gpurun_out/r5a/pmc [name-substring]
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
        vals[(nm, r.get("Grid_Size", ""))][r["Counter_Name"]].append(float(r["Counter_Value"]))
print(f"{'kernel':60s} {'grid':>8s} {'VALU busy':>9s} {'active':>7s} {'stall':>7s} {'wait':>7s} {'FETCH MB':>9s} {'WRITE MB':>9s}")
for (nm, grid), cs in sorted(vals.items()):
    a = {k: sum(v) / len(v) for k, v in cs.items()}
    if "GRBM_GUI_ACTIVE" not in a or "SQ_INSTS_VALU" not in a:
        continue
    cyc = a["GRBM_GUI_ACTIVE"] / 8
    valu = a["SQ_INSTS_VALU"] * 2 / 1024 / cyc
    wc = a.get("SQ_WAVE_CYCLES", 0) or 1
    print(f"{nm[:60]:60s} {grid:>8s} {valu:9.2f} {a.get('SQ_ACTIVE_INST_ANY', 0) / wc:7.2f} "
          f"{a.get('SQ_WAIT_INST_ANY', 0) / wc:7.2f} {a.get('SQ_WAIT_ANY', 0) / wc:7.2f} "
          f"{a.get('FETCH_SIZE', 0) / 1024:9.1f} {a.get('WRITE_SIZE', 0) / 1024:9.1f}")
