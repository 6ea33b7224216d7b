#!/bin/bash
# tests + A/B bench variants (env assignments per variant) + one rocprof kernel-stats pass
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-ab}
mkdir -p "$OUT"
ROOTDIR=$(pwd)
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -m pytest $TESTS -q -x > "$OUT/tests.log" 2>&1
  rc=$?; echo "tests rc=$rc" | tee -a "$OUT/status"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
i=0
for v in ${VARIANTS:-base}; do
  i=$((i+1))
  if [ "$v" = "base" ]; then envs=""; else envs="$v"; fi
  env $envs timeout -k 10 400 python bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err"
  rc=$?; echo "bench $v rc=$rc $(cat $OUT/bench_$i.json | head -c 200)" | tee -a "$OUT/status"
  [ $rc -ne 0 ] && exit $rc
done
if [ "${PROF:-1}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOTDIR/$OUT/prof" -o run -- python3 "$ROOTDIR/bench.py" --steps 3 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > "$ROOTDIR/$OUT/prof_bench.json" 2> "$ROOTDIR/$OUT/prof.err"
  rc=$?; echo "rocprof rc=$rc" | tee -a "$ROOTDIR/$OUT/status"
  exit $rc
fi
exit 0
