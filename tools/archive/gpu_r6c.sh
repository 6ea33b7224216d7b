#!/bin/bash
# round 3 (late): inner BatchNorm backward statistics from the data gradient's GEMM epilogue / split-K finish
# (SV_EPI_STORE_BN_BWD, sv_gemm_slab_finish_bn_bwd): full -m gpu suite, then the classification step A/B
# against the split-K finish only (SV_BN_BWD_EPI=split) and the separate statistics pass (0), interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r6c}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_resnet_gpu.py tests/test_resnet_parity_256_gpu.py tests/test_golden_gpu.py > "$OUT/gpu_tests.txt" 2>&1
rc=$?; echo "gpu tests rc=$rc $(tail -1 $OUT/gpu_tests.txt)"; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
  for e in 1 split 0; do
    SV_BN_BWD_EPI=$e timeout -k 10 300 python bench.py --workload classification --steps 30 --warmup 5 --no-cpu-baseline > "$OUT/bench_e${e}_$r.json" 2> "$OUT/bench_e${e}_$r.err"
    rc=$?; echo "bench epi=$e r$r rc=$rc $(grep -o '"value": [0-9.]*' $OUT/bench_e${e}_$r.json)"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
