"""Per-kernel launch durations from a rocprofv3 kernel trace, grouped by (kernel, grid size):
    python tools/trace_by_grid.py <run_kernel_trace.csv> <kernel substring> [...]"""
import csv
import sys
from collections import defaultdict

path, pats = sys.argv[1], sys.argv[2:]
groups = defaultdict(list)
for r in csv.DictReader(open(path)):
    name = r["Kernel_Name"]
    if not any(p in name for p in pats):
        continue
    key = (name[:70], int(r["Grid_Size_X"]) // max(int(r["Workgroup_Size_X"]), 1), int(r["Grid_Size_Y"]),
           int(r["Grid_Size_Z"]), r["Queue_Id"])
    groups[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
    v.sort()
    print(f"{k[0]:70s} wg={k[1]:6d} y={k[2]:3d} z={k[3]:3d} q={k[4]} n={len(v):4d} "
          f"mean={sum(v) / len(v):8.1f}us med={v[len(v) // 2]:8.1f} min={v[0]:8.1f} tot={sum(v) / 1e3:7.2f}ms")
