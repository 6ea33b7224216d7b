#!/bin/bash
# round 5: HIP API statistics of the eval forward and the training step (where the copyBuffer launches come from)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOTDIR=$(pwd)
N=${1:-r11y}
O=gpurun_out/$N
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for w in inf train; do
  A=$([ $w = inf ] && echo --inference || echo "")
  timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d "$ROOTDIR/$O/$w" -o run -- python3 "$ROOTDIR/bench.py" $A --steps 5 --warmup 2 --no-cpu-baseline > "$ROOTDIR/$O/$w.json" 2> "$ROOTDIR/$O/$w.err" || { tail -20 "$ROOTDIR/$O/$w.err"; exit 1; }
  cd "$ROOTDIR"
  python - "$O/$w" <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
st = glob.glob(d + "/**/*hip_api_stats.csv", recursive=True)
if st:
    rows = list(csv.DictReader(open(st[0])))
    rows.sort(key=lambda r: -int(r["Calls"]))
    for r in rows[:25]:
        print(r["Name"], r["Calls"], r.get("TotalDurationNs"))
tr = glob.glob(d + "/**/*hip_api_trace.csv", recursive=True)
kt = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)
if tr and kt:
    api = list(csv.DictReader(open(tr[0])))
    ks = list(csv.DictReader(open(kt[0])))
    # the kernel launched just before each copyBuffer on the same stream
    ks.sort(key=lambda r: int(r["Start_Timestamp"]))
    prev = collections.Counter()
    last = {}
    for r in ks:
        q = r.get("Stream_Id", r.get("Queue_Id", "0"))
        n = r["Kernel_Name"][:90]
        if "copyBuffer" in n:
            prev[last.get(q, "?")] += 1
        last[q] = n
    print("kernel before copyBuffer:")
    for k, v in prev.most_common(12):
        print(v, k)
    mc = collections.Counter()
    for r in api:
        if "Memcpy" in r["Function"] or "Memset" in r["Function"]:
            mc[r["Function"]] += 1
    print("memcpy/memset api:", dict(mc))
PY
  find "$ROOTDIR/$O/$w" -name "*trace.csv" -delete
  cd /tmp
done
