"""Per-kernel (and, with --shapes, per kernel x grid) time per step from a rocprofv3 kernel_trace.csv.

    python tools/trace_summary.py run_kernel_trace.csv STEPS [TOP] [--shapes] [--match SUBSTR]
"""
import collections
import csv
import re
import sys

path, steps = sys.argv[1], float(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 and sys.argv[3].isdigit() else 30
match = sys.argv[sys.argv.index("--match") + 1] if "--match" in sys.argv else None
by_name = collections.defaultdict(lambda: [0, 0.0])
by_shape = collections.defaultdict(lambda: [0, 0.0])
for r in csv.DictReader(open(path)):
    nm = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
    dt = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3  # us
    by_name[nm][0] += 1
    by_name[nm][1] += dt
    wg = int(r["Workgroup_Size_X"]) or 1
    key = (nm, int(r["Grid_Size_X"]) // wg, int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]))
    by_shape[key][0] += 1
    by_shape[key][1] += dt
tot = sum(v[1] for v in by_name.values())
print(f"total kernel time per step: {tot / steps / 1e3:.2f} ms over {sum(v[0] for v in by_name.values()) / steps:.0f} launches")
for nm, (n, t) in sorted(by_name.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"{t / tot * 100:6.2f}% {t / steps / 1e3:7.2f} ms/step n={n / steps:6.1f} avg={t / n:8.1f} us  {nm[:90]}")
if "--shapes" in sys.argv:
    print()
    for (nm, gx, gy, gz), (n, t) in sorted(by_shape.items(), key=lambda kv: -kv[1][1])[:top * 2]:
        if match and match not in nm:
            continue
        print(f"{t / steps:9.1f} us/step n={n / steps:4.1f} avg={t / n:8.1f} us wgs=({gx},{gy},{gz}) {nm[:70]}")
