#!/bin/bash
# ResNet / classification iteration on the GPU box: tests, one bench line, one rocprof kernel-stats pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-cls}
mkdir -p "$OUT"
ROOTDIR=$(pwd)
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_resnet_gpu.py tests/test_trainer_gpu.py} -q -x --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $OUT/tests.log)"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --workload classification --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc $(head -c 260 $OUT/bench.json)"
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOTDIR/$OUT/prof" -o run -- python3 "$ROOTDIR/bench.py" --workload classification --steps 3 --warmup 2 --no-cpu-baseline > "$ROOTDIR/$OUT/prof_bench.json" 2> "$ROOTDIR/$OUT/prof.err"
rc=$?; echo "rocprof rc=$rc"
exit $rc
