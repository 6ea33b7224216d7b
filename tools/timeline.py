"""Per-step timeline of a rocprofv3 kernel trace: step boundaries at the AdamW launches, per-queue busy
time, the union of busy time, and the forward / backward split (first backward kernel = the first
kernel on a second queue, or the first `_bwd` / `dgrad` launch after the step start).

    python tools/timeline.py run_kernel_trace.csv
"""
import csv
import re
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    nm = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]), nm))
rows.sort()
ad = [i for i, r in enumerate(rows) if "adamw" in r[3]]
for a, b in zip(ad, ad[1:]):
    seg = rows[a + 1:b + 1]
    t0, t1 = seg[0][0], seg[-1][1]
    busy = {}
    for s, e, q, _ in seg:
        busy[q] = busy.get(q, 0) + (e - s)
    iv = sorted((s, e) for s, e, _, _ in seg)
    union, cs, ce = 0, iv[0][0], iv[0][1]
    for s, e in iv[1:]:
        if s > ce:
            union += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    union += ce - cs
    # forward ends at the pool/LN forward kernel
    fwd_end = next((e for s, e, q, n in seg if "pool_ln_fwd" in n), None)
    print(f"step {t1 - t0:9.0f} ns -> {(t1 - t0) / 1e6:.2f} ms | union busy {union / 1e6:.2f} ms | "
          + " ".join(f"q{q}:{v / 1e6:.2f}" for q, v in sorted(busy.items()))
          + (f" | fwd {(fwd_end - t0) / 1e6:.2f} ms, bwd+opt {(t1 - fwd_end) / 1e6:.2f} ms" if fwd_end else ""))
