#!/bin/bash
# merged weight-gradient folds: kernel + ConvNeXt parity tests, then interleaved step A/B (SV_MERGED_FOLDS)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r4j}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_parity_geometry_gpu.py tests/test_backbone_gpu.py tests/test_golden_gpu.py -k "reduce or convnext or golden or backbone" > "$OUT/tests.log" 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $OUT/tests.log)"
[ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" "$OUT/tests.log" | head -20; exit $rc; }
for r in 1 2 3; do
  for v in 1 0; do
    SV_MERGED_FOLDS=$v SV_BENCH_PROBE=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/b_${v}_$r.json" 2>"$OUT/b_${v}_$r.err"
    echo "merged=$v run $r rc=$? $(python -c "import json;print(json.load(open('$OUT/b_${v}_$r.json'))['value'])" 2>/dev/null)"
  done
done
exit 0
