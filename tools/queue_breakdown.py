"""Per-queue kernel time of one step (the last full step between two AdamW launches) of a rocprofv3
kernel trace, by kernel family: which stream carries the critical path and what fills it.
    python tools/queue_breakdown.py <run_kernel_trace.csv> [top]"""
import csv
import re
import sys
from collections import defaultdict

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    nm = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]), nm))
rows.sort()
top = int(sys.argv[2]) if len(sys.argv) > 2 else 14
ad = [i for i, r in enumerate(rows) if "adamw" in r[3]]
seg = rows[ad[-2] + 1:ad[-1] + 1]
byq = defaultdict(lambda: defaultdict(lambda: [0.0, 0]))
for s, e, q, n in seg:
    key = n if "gemm" in n else n.split("<")[0]
    byq[q][key][0] += (e - s) / 1e3
    byq[q][key][1] += 1
print(f"step {(seg[-1][1] - seg[0][0]) / 1e3:.0f} us")
for q in sorted(byq):
    tot = sum(v[0] for v in byq[q].values())
    print(f"queue {q}: {tot:.0f} us in {sum(v[1] for v in byq[q].values())} launches")
    for k, (v, c) in sorted(byq[q].items(), key=lambda kv: -kv[1][0])[:top]:
        print(f"   {v:8.0f} us {c:4d}x  {k[:110]}")
