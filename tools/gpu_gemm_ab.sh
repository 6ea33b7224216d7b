#!/bin/bash
# GEMM implementation A/B: correctness of the forced implementation, then standalone shape timings
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-gab}
mkdir -p "$OUT"
for impl in ${IMPLS:-8}; do
  SV_GEMM_IMPL=$impl timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "gemm or wgrad or stem or layerscale" > "$OUT/tests_$impl.log" 2>&1
  rc=$?; echo "impl $impl tests rc=$rc $(tail -1 $OUT/tests_$impl.log)"
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
done
for impl in 0 ${IMPLS:-8}; do
  SV_GEMM_IMPL=$impl timeout -k 10 300 python tools/gemm_bench.py --stages ${STAGES:-S1,S2,S3,S4} --iters 20 ${GB_ARGS:-} > "$OUT/bench_$impl.log" 2>&1
  rc=$?; echo "impl $impl bench rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
