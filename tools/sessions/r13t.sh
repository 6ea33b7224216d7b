#!/bin/bash
# round 6: matrix-core depthwise weight gradient with the conflict-free dz fill: parity + standalone timing + SQ split
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOTDIR=$(pwd)
N=${1:-r13t}
O=$ROOTDIR/gpurun_out/$N
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_dw_mfma_gpu.py -k weight_gradient > $O/dwm.log 2>&1 || { grep -E "FAIL|Error|assert" $O/dwm.log | head -20; tail -20 $O/dwm.log; exit 1; }
grep -E "passed|failed" $O/dwm.log
timeout -k 10 300 python -u tools/dw_bench.py --iters 20 > $O/dw_bench.txt 2>&1 || { tail -20 $O/dw_bench.txt; exit 1; }
grep -E "wgrad" $O/dw_bench.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --output-format csv -d "$O/pmc_sq" -o run -- python3 "$ROOTDIR/tools/dw_bench.py" --stages S3 --iters 2 > "$O/pmc_sq.log" 2>&1 || { tail -5 "$O/pmc_sq.log"; exit 1; }
cd "$ROOTDIR"
python - $O/pmc_sq > $O/wgrad_sq.txt <<'PYEOF'
import collections, csv, glob, re, sys
v = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        nm = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
        if "wgrad" not in nm:
            continue
        v[(nm[:60], r["Grid_Size"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, dd in sorted(v.items()):
    print(k[0], "grid", k[1])
    for c, xs in sorted(dd.items()):
        print(f"    {c:28s} {sum(xs) / len(xs):16.1f}")
PYEOF
cat $O/wgrad_sq.txt
