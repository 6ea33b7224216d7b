#!/bin/bash
# round 3: ResNet-50 classification step budget — kernel traces with the side stream on and off
# (off: every kernel alone, so the trace is the step's serial kernel budget)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r4k}
mkdir -p "$OUT"
ROOTDIR=$(pwd)
cd /tmp && export TMPDIR=/tmp
for side in 1 0; do
  SV_SIDE_STREAM=$side timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOTDIR/$OUT/prof_side$side" -o run -- python3 "$ROOTDIR/bench.py" --workload classification --steps 3 --warmup 3 --no-cpu-baseline > "$ROOTDIR/$OUT/prof_side$side.json" 2> "$ROOTDIR/$OUT/prof_side$side.err"
  rc=$?; echo "rocprof side=$side rc=$rc $(head -c 120 $ROOTDIR/$OUT/prof_side$side.json)"; [ $rc -ne 0 ] && exit $rc
done
cd "$ROOTDIR"
for side in 1 0; do
  SV_SIDE_STREAM=$side timeout -k 10 300 python bench.py --workload classification --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_side$side.json" 2> "$OUT/bench_side$side.err"
  rc=$?; echo "bench side=$side rc=$rc $(head -c 120 $OUT/bench_side$side.json)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
