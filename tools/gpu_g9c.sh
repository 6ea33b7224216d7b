#!/bin/bash
# v9 iteration: family parity, standalone GEMM timings (STAGES/CASES), two bench lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-g9c}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_family_gpu.py ${EXTRA_TESTS:-} > "$OUT/tests.log" 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $OUT/tests.log)"
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" "$OUT/tests.log" | head -20; exit $rc; }
timeout -k 10 400 python -u tools/gemm_bench.py --stages ${STAGES:-S1,S2,S3,S4} --iters 20 --impls 0 --cases ${CASES:-fc} > "$OUT/gemm.txt" 2> "$OUT/gemm.err"
rc=$?; echo "gemm rc=$rc"; grep -v torch "$OUT/gemm.txt"
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench$i.json" 2> "$OUT/bench$i.err"
  rc=$?; echo "bench rc=$rc $(python3 -c "import json; d=json.load(open('$OUT/bench$i.json')); print(d['value'], d['ms_per_step'])")"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
