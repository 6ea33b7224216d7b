#!/bin/bash
# round 3 (late): the ResNet stem forward on the gathered v3 GEMM over 8-channel pixels (mode 6): ResNet tests,
# stem conv timing, classification A/B against the register-staged stem (SV_STEM_GATHER=0)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r6k}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_resnet_gpu.py tests/test_resnet_parity_256_gpu.py tests/test_golden_gpu.py tests/test_trainer_gpu.py > "$OUT/gpu_tests.txt" 2>&1
rc=$?; echo "gpu tests rc=$rc $(tail -1 $OUT/gpu_tests.txt)"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/conv_bench.py --only stem > "$OUT/conv_stem.txt" 2>&1
rc=$?; echo "stem $(grep stem $OUT/conv_stem.txt)"; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then export SV_STEM_GATHER=0; else unset SV_STEM_GATHER; fi
    timeout -k 10 300 python bench.py --workload classification --steps 30 --warmup 5 --no-cpu-baseline > "$OUT/bench_${v}_$r.json" 2> "$OUT/bench_${v}_$r.err"
    rc=$?; echo "bench $v r$r rc=$rc $(grep -o '"value": [0-9.]*' $OUT/bench_${v}_$r.json)"; [ $rc -ne 0 ] && exit $rc
  done
done
unset SV_STEM_GATHER
exit 0
