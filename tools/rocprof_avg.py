"""Per-class average launch duration from a rocprofv3 ``--stats`` kernel_stats.csv, for bench.py's rocprof-derived
roofline fraction (the line carries the profiler's figure beside the HIP-event probe's).

    python tools/rocprof_avg.py <kernel_stats.csv> <config key, e.g. convnext_base/512/bs32/bf16> <source tag>

Classes use the kernel-name matches of profiles/traffic.json (the PMC classes, tools/pmc_classes.py), so the average
is over the same launches the traffic figure counts.  Merges into profiles/rocprof_avg.json."""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
path, key, source = sys.argv[1], sys.argv[2], sys.argv[3]
traffic = json.load(open(os.path.join(ROOT, "profiles", "traffic.json")))["configs"][key]
rows = list(csv.DictReader(open(path)))
out_path = os.path.join(ROOT, "profiles", "rocprof_avg.json")
doc = json.load(open(out_path)) if os.path.exists(out_path) else {
    "note": "rocprofv3 --kernel-trace --stats average launch duration per probed kernel class (the kernel-name matches "
            "of traffic.json), per configuration; bench.py reports roofline.frac_rocprof = roof time per launch "
            "(the probe's algorithmic bytes / FLOPs) / this average.  Written by tools/rocprof_avg.py.",
    "configs": {}}
cfg = doc["configs"].setdefault(key, {})
for cls in ("wgrad", "fc2_dgrad", "dgrad", "fwd"):
    det = traffic.get(f"{cls}_detail")
    if not det:
        continue
    pats = [m[0] for m in det["kernel_match"]]
    calls, ns = 0, 0.0
    for r in rows:
        if any(p in r["Name"] for p in pats):
            calls += int(r["Calls"])
            ns += float(r["TotalDurationNs"])
    if calls:
        cfg[cls] = {"avg_launch_us": round(ns / calls / 1e3, 2), "calls": calls, "kernel_match": pats, "source": source}
json.dump(doc, open(out_path, "w"), indent=1)
print(json.dumps(cfg, indent=1))
