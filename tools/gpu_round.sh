#!/bin/bash
# GPU-box driver for one measurement round: tests, smoke, bench, rocprof stats, PMC traffic passes.
# Stops at the first step that crashes/faults/times out (exit codes other than 0 or 1 for pytest).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r}
mkdir -p "$OUT"
STEPS=${STEPS:-10}
ROOTDIR=$(pwd)
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
  rc=$?; echo "tests rc=$rc" | tee -a "$OUT/status"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  rc=$?; echo "smoke rc=$rc" | tee -a "$OUT/status"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
timeout -k 10 900 python bench.py --steps $STEPS --warmup 3 ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc" | tee -a "$OUT/status"
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOTDIR/$OUT/prof" -o run -- python3 "$ROOTDIR/bench.py" --steps 3 --warmup 2 --no-cpu-baseline > "$ROOTDIR/$OUT/prof_bench.json" 2> "$ROOTDIR/$OUT/prof.err"
rc=$?; echo "rocprof rc=$rc" | tee -a "$ROOTDIR/$OUT/status"
[ $rc -ne 0 ] && exit $rc
if [ "${PMC:-1}" = "1" ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 900 rocprofv3 --kernel-trace --pmc $c --output-format csv -d "$ROOTDIR/$OUT/pmc_$c" -o run -- python3 "$ROOTDIR/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$ROOTDIR/$OUT/pmc_$c.json" 2> "$ROOTDIR/$OUT/pmc_$c.err"
    rc=$?; echo "pmc $c rc=$rc" | tee -a "$ROOTDIR/$OUT/status"
    [ $rc -ne 0 ] && exit $rc
  done
fi
exit 0
