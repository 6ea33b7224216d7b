#!/bin/bash
# round 3 (late): a projection-shortcut block's two output BatchNorm backwards in one statistics and one apply
# pass (sv_bn_bwd_*_dual): ResNet parity tests, then the classification step A/B against SV_BN_DUAL=0, interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r6f}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_resnet_gpu.py tests/test_resnet_parity_256_gpu.py tests/test_golden_gpu.py tests/test_trainer_gpu.py > "$OUT/gpu_tests.txt" 2>&1
rc=$?; echo "gpu tests rc=$rc $(tail -1 $OUT/gpu_tests.txt)"; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
  for e in 1 0; do
    SV_BN_DUAL=$e timeout -k 10 300 python bench.py --workload classification --steps 30 --warmup 5 --no-cpu-baseline > "$OUT/bench_d${e}_$r.json" 2> "$OUT/bench_d${e}_$r.err"
    rc=$?; echo "bench dual=$e r$r rc=$rc $(grep -o '"value": [0-9.]*' $OUT/bench_d${e}_$r.json)"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
