#!/bin/bash
# round 6 profile: (1) the default training step under the kernel tracer (per-kernel stats, main / side queue
# breakdown); (2) PMC passes over the depthwise kernels at S3 and S1 (dw_bench): HBM bytes (FETCH_SIZE, WRITE_SIZE in
# separate passes) and the SQ wave-cycle split (waits, LDS bank conflicts, VALU / MFMA busy) -- VALU ring kernels
# beside the matrix-core ones
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOTDIR=$(pwd)
N=${1:-r13h}
O=$ROOTDIR/gpurun_out/$N
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 "$ROOTDIR/bench.py" --steps 3 --warmup 2 --no-cpu-baseline > "$O/prof_bench.json" 2> "$O/prof.err" || { tail -20 "$O/prof.err"; exit 1; }
for pass in FETCH_SIZE WRITE_SIZE "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY"; do
  tag=$(echo $pass | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d "$O/pmc_$tag" -o run -- python3 "$ROOTDIR/tools/dw_bench.py" --stages S3,S1 --iters 2 > "$O/pmc_$tag.log" 2>&1 || { tail -5 "$O/pmc_$tag.log"; exit 1; }
done
cd "$ROOTDIR"
KT=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python tools/queue_breakdown.py $KT 30 > $O/queues.txt && head -60 $O/queues.txt
ST=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python tools/stats_md.py $ST 5 "round 6 $N" "rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline" 40 > $O/kernel_stats.md
python tools/pmc_traffic_by_kernel.py $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE dwconv > $O/dw_traffic.txt; python tools/pmc_traffic_by_kernel.py $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE dw7 >> $O/dw_traffic.txt; cat $O/dw_traffic.txt
python - $O/pmc_SQ_WAVE_CYCLES > $O/dw_sq.txt <<'PYEOF'
import collections, csv, glob, re, sys
v = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        nm = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
        if "dw" not in nm:
            continue
        v[(nm[:60], r["Grid_Size"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(v.items()):
    print(k[0], "grid", k[1])
    for c, xs in sorted(d.items()):
        print(f"    {c:28s} {sum(xs) / len(xs):16.1f}")
PYEOF
cat $O/dw_sq.txt | head -60
gzip -f $KT
