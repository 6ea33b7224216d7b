#!/bin/bash
# depthwise kernels: parity tests, standalone timings, two bench lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-dw}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread ${TESTS:-tests/test_kernels_gpu.py} -k "dwconv or backbone" > "$OUT/tests.log" 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $OUT/tests.log)"
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" "$OUT/tests.log" | head -20; exit $rc; }
timeout -k 10 300 python tools/dw_bench.py > "$OUT/dw.txt" 2>&1
rc=$?; echo "dw rc=$rc"; grep -v amdgpu "$OUT/dw.txt"
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench$i.json" 2> "$OUT/bench$i.err"
  rc=$?; echo "bench rc=$rc $(python3 -c "import json; d=json.load(open('$OUT/bench$i.json')); print(d['value'], d['ms_per_step'])")"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
