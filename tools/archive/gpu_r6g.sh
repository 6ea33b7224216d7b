#!/bin/bash
# round 3 final tree after the BatchNorm fusions: full -m gpu suite + smoke, classification line, and the
# classification serial kernel budget (side stream off) under rocprofv3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r6g}
mkdir -p "$OUT"
ROOTDIR=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $OUT/tests.log)"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 $OUT/smoke.txt)"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --workload classification --steps 30 --warmup 5 --no-cpu-baseline > "$OUT/bench_cls.json" 2> "$OUT/bench_cls.err"
rc=$?; echo "cls rc=$rc $(grep -o '"value": [0-9.]*' $OUT/bench_cls.json)"; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
SV_SIDE_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOTDIR/$OUT/prof_side0" -o run -- python3 "$ROOTDIR/bench.py" --workload classification --steps 3 --warmup 3 --no-cpu-baseline > "$ROOTDIR/$OUT/prof_side0.json" 2> "$ROOTDIR/$OUT/prof_side0.err"
rc=$?; echo "rocprof rc=$rc"
exit $rc
