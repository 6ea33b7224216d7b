#!/bin/bash
# round 3 (late): ResNet-50 classification serial kernel budget on the final tree — one kernel trace with the
# side stream off (every kernel alone) and the standalone conv pass timings
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r6a}
mkdir -p "$OUT"
ROOTDIR=$(pwd)
timeout -k 10 300 python tools/conv_bench.py --iters 20 > "$OUT/conv_bench.txt" 2>&1
rc=$?; echo "conv_bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
SV_SIDE_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOTDIR/$OUT/prof_side0" -o run -- python3 "$ROOTDIR/bench.py" --workload classification --steps 3 --warmup 3 --no-cpu-baseline > "$ROOTDIR/$OUT/prof_side0.json" 2> "$ROOTDIR/$OUT/prof_side0.err"
rc=$?; echo "rocprof rc=$rc $(head -c 120 $ROOTDIR/$OUT/prof_side0.json)"
exit $rc
