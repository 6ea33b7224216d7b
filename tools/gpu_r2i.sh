#!/bin/bash
# lean-mode per-batch release of side-stream operands: GEMM family / golden / ConvNeXt backward tests,
# then ConvNeXt-large bs64 twice back to back (reserved memory, alloc retries, run-to-run spread) and
# the base bs32 headline line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r2i}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gemm_family_gpu.py \
  tests/test_golden_r2_gpu.py tests/test_parity_geometry_gpu.py tests/test_backbone_gpu.py tests/test_resnet_gpu.py \
  > "$OUT/tests.log" 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $OUT/tests.log)"
[ $rc -gt 1 ] && exit $rc
for i in 1 2; do
  timeout -k 10 400 python bench.py --backbone convnext_large --batch 64 --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/large$i.json" 2> "$OUT/large$i.err"
  rc=$?; echo "large$i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/base.json" 2> "$OUT/base.err"
rc=$?; echo "base rc=$rc"
exit $rc
