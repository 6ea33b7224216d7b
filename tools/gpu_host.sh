#!/bin/bash
# host enqueue vs device time per step (both workloads), then the two bench lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-host}
mkdir -p "$OUT"
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q -rf --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
  rc=$?; echo "tests rc=$rc $(tail -1 $OUT/tests.log)"
  [ $rc -ne 0 ] && exit $rc
fi
for w in classification localization; do
  timeout -k 10 300 python tools/host_time.py --workload $w > "$OUT/host_$w.log" 2>&1
  rc=$?; echo "host $w rc=$rc $(grep host "$OUT/host_$w.log" | tail -1)"
  [ $rc -ne 0 ] && exit $rc
  timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err"
  rc=$?; echo "bench $w rc=$rc $(head -c 200 "$OUT/bench_$w.json" | sed 's/.*"value": \([0-9.]*\).*/\1/')"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
