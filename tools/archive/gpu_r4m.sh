#!/bin/bash
# round 3: BN finish (128 partial streams per 32 channels) + in-place masked block gradient:
# BN / ResNet / trainer tests, classification bench, kernel trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r4m}
mkdir -p "$OUT"
ROOTDIR=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_resnet_gpu.py tests/test_resnet_parity_256_gpu.py tests/test_trainer_gpu.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $OUT/tests.log)"; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" "$OUT/tests.log" | head -20; exit $rc; }
for r in 1 2; do
  timeout -k 10 300 python bench.py --workload classification --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/cls_$r.json" 2> "$OUT/cls_$r.err"
  rc=$?; echo "cls $r rc=$rc $(python -c "import json;d=json.load(open('$OUT/cls_$r.json'));print(d['value'], d['ms_per_step'])" 2>/dev/null)"; [ $rc -ne 0 ] && exit $rc
done
cd /tmp && export TMPDIR=/tmp
SV_SIDE_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOTDIR/$OUT/prof_side0" -o run -- python3 "$ROOTDIR/bench.py" --workload classification --steps 3 --warmup 3 --no-cpu-baseline > "$ROOTDIR/$OUT/prof_side0.json" 2> "$ROOTDIR/$OUT/prof_side0.err"
rc=$?; echo "rocprof rc=$rc"
exit $rc
