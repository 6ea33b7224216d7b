"""Idle gaps of the main queue within one step of a rocprofv3 kernel trace (the last full step between two AdamW
launches): every gap longer than a threshold, the main-queue kernels on either side and what the other queues ran
during it -- where the critical path waits.
    python tools/queue_gaps.py <run_kernel_trace.csv> [min_gap_us] [main_queue_id]"""
import csv
import re
import sys
from collections import defaultdict

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    nm = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]), nm))
rows.sort()
thr = float(sys.argv[2]) if len(sys.argv) > 2 else 20.0
ad = [i for i, r in enumerate(rows) if "adamw" in r[3]]
seg = rows[ad[-2] + 1:ad[-1] + 1]
main_q = int(sys.argv[3]) if len(sys.argv) > 3 else seg[-1][2]  # the queue AdamW runs on
main = [r for r in seg if r[2] == main_q]
other = [r for r in seg if r[2] != main_q]
t0 = seg[0][0]
tot_gap, by_next = 0.0, defaultdict(float)
print(f"step {(seg[-1][1] - t0) / 1e3:.0f} us, main queue {main_q}: {len(main)} launches")
busy = 0
end = main[0][0]
for i, (s, e, q, n) in enumerate(main):
    gap = (s - end) / 1e3
    if gap > 0:
        tot_gap += gap
    if gap > thr:
        during = [o[3].split("<")[0][:40] for o in other if o[0] < s and o[1] > end]
        prev = main[i - 1][3].split("<")[0][:40] if i else "-"
        print(f"  +{(end - t0) / 1e3:8.1f} us  gap {gap:7.1f} us  {prev:40s} -> {n.split('<')[0][:40]:40s}  other: "
              f"{', '.join(sorted(set(during)))[:90]}")
        by_next[n.split("<")[0][:60]] += gap
    busy += (e - s) / 1e3
    end = max(end, e)
print(f"main busy {busy:.0f} us, idle {tot_gap:.0f} us")
for k, v in sorted(by_next.items(), key=lambda kv: -kv[1])[:12]:
    print(f"   {v:8.1f} us before {k}")
