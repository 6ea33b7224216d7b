#!/bin/bash
# ResNet iteration: conv/BN/trainer/geometry parity tests, conv pass timings, classification bench x2
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-clsq}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_resnet_gpu.py tests/test_trainer_gpu.py tests/test_parity_geometry_gpu.py -q -x --timeout 120 --timeout-method thread -k "${TK:-not convnext}" > "$OUT/tests.log" 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $OUT/tests.log)"
[ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" "$OUT/tests.log" | head -20; exit $rc; }
timeout -k 10 120 python tools/conv_bench.py > "$OUT/conv.txt" 2>&1 || exit $?
cat "$OUT/conv.txt" | grep -v amdgpu
for r in 1 2; do
  timeout -k 10 300 python bench.py --workload classification --steps 30 --warmup 5 --no-cpu-baseline > "$OUT/bench_$r.json" 2> "$OUT/bench_$r.err"
  rc=$?; echo "r=$r rc=$rc $(python3 -c "import json; d=json.load(open('$OUT/bench_$r.json')); print(d['value'], d['ms_per_step'])" 2>&1 | tail -1)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
