#!/bin/bash
# LayerNorm kernel tests + one ConvNeXt-large bs64 bench line (configs[4] shape, 1 GPU)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-large}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "layernorm" -q -x --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $OUT/tests.log)"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --backbone convnext_large --batch 64 --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/large.json" 2> "$OUT/large.err"
rc=$?; echo "large rc=$rc $(head -c 240 $OUT/large.json)"
exit $rc
