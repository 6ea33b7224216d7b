#!/bin/bash
# round measurement set: full GPU suite, the default bench line (with cpu_baseline), rocprof kernel
# stats, PMC FETCH_SIZE / WRITE_SIZE passes (separate runs) over a short bench, classification line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r3m}
mkdir -p "$OUT"
ROOTDIR=$(pwd)
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
  rc=$?; echo "tests rc=$rc $(tail -1 $OUT/tests.log)"
  [ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" "$OUT/tests.log" | head -20; exit $rc; }
fi
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc $(head -c 300 $OUT/bench.json)"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --workload classification --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench_cls.json" 2> "$OUT/bench_cls.err"
rc=$?; echo "cls rc=$rc $(head -c 200 $OUT/bench_cls.json)"
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOTDIR/$OUT/prof" -o run -- python3 "$ROOTDIR/bench.py" --steps 3 --warmup 2 --no-cpu-baseline > "$ROOTDIR/$OUT/prof_bench.json" 2> "$ROOTDIR/$OUT/prof.err"
rc=$?; echo "rocprof rc=$rc"
[ $rc -ne 0 ] && exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $c --output-format csv -d "$ROOTDIR/$OUT/pmc_$c" -o run -- python3 "$ROOTDIR/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$ROOTDIR/$OUT/pmc_$c.log" 2>&1
  rc=$?; echo "pmc $c rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
