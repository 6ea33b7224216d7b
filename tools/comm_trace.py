"""Which kernels ran while a comm-stream proxy waited (tests/test_comm_reserve_gpu.py under rocprofv3 --kernel-trace).

    python tools/comm_trace.py comm_kernel_trace.csv --queue 4 --skip 23 --launch 32,36,4

--queue: the comm stream's hardware queue (the one holding only the proxy reductions and timing fills);
--skip: proxy launches before the hooked step (the standalone timing loop: 3 + 20); --launch: hook indices the
test printed as worst.  Lists every other queue's kernels overlapping the 0.9 ms before each proxy's end.
"""
import argparse
import csv
import re
from collections import Counter, defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--queue", type=int, required=True)
ap.add_argument("--skip", type=int, default=23)
ap.add_argument("--launch", default="0")
ap.add_argument("--window-us", type=float, default=900.0)
a = ap.parse_args()
rows = []
for r in csv.DictReader(open(a.trace)):
    nm = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]), nm[:58], r["Grid_Size_X"]))
rows.sort()
byq = defaultdict(Counter)
for s, e, q, n, g in rows:
    byq[q][n] += 1
for q, c in sorted(byq.items()):
    print(f"queue {q}: {sum(c.values())} kernels, top: " + "; ".join(f"{n} x{k}" for n, k in c.most_common(3)))
prox = [r for r in rows if r[2] == a.queue and "reduce_kernel" in r[3]]
for idx in [int(x) for x in a.launch.split(",")]:
    s, e, q, n, g = prox[a.skip + idx]
    print(f"== hook launch #{idx}: proxy ran {(e - s) / 1e3:.1f} us (times below relative to its start)")
    for r in rows:
        if r[2] != a.queue and r[1] > s - a.window_us * 1e3 and r[0] < e:
            print(f"    q{r[2]} {(r[0] - s) / 1e3:9.1f} .. {(r[1] - s) / 1e3:9.1f} us  {r[3]}  grid {r[4]}")
