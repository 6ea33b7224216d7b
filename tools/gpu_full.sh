#!/bin/bash
# full GPU suite, one bench line, rocprof kernel stats of a short bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-full}
mkdir -p "$OUT"
ROOTDIR=$(pwd)
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
  rc=$?; echo "tests rc=$rc $(tail -1 $OUT/tests.log)"
  [ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" "$OUT/tests.log" | head -20; exit $rc; }
fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc $(head -c 400 $OUT/bench.json)"
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOTDIR/$OUT/prof" -o run -- python3 "$ROOTDIR/bench.py" --steps 3 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > "$ROOTDIR/$OUT/prof_bench.json" 2> "$ROOTDIR/$OUT/prof.err"
rc=$?; echo "rocprof rc=$rc"
exit $rc
