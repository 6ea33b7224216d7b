#!/bin/bash
# quick GPU iteration: selected tests (TESTS), then one bench line (+ optional rocprof kernel stats)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-q}
mkdir -p "$OUT"
ROOTDIR=$(pwd)
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q -rf --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
  rc=$?; echo "tests rc=$rc $(tail -1 $OUT/tests.log)"
  [ $rc -ne 0 ] && exit $rc
fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
  rc=$?; echo "bench rc=$rc $(head -c 300 $OUT/bench.json)"
  [ $rc -ne 0 ] && exit $rc
fi
if [ "${PROF:-0}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOTDIR/$OUT/prof" -o run -- python3 "$ROOTDIR/bench.py" --steps 3 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > "$ROOTDIR/$OUT/prof_bench.json" 2> "$ROOTDIR/$OUT/prof.err"
  rc=$?; echo "rocprof rc=$rc"
  exit $rc
fi
exit 0
