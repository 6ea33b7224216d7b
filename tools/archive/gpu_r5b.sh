#!/bin/bash
# round 3, session 3: packed-FMA depthwise kernels (parity tests, standalone A/B against the scalar build,
# interleaved bench lines) and the store-shape microbenchmark for the v9 epilogue
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r5b}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_backbone_gpu.py tests/test_parity_geometry_gpu.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $OUT/tests.log)"; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" "$OUT/tests.log" | head -20; exit $rc; }
timeout -k 10 120 ./tools/store_shape > "$OUT/store_shape.txt" 2>&1
rc=$?; echo "store_shape rc=$rc"; cat "$OUT/store_shape.txt"; [ $rc -ne 0 ] && exit $rc
for v in pk scalar; do
  if [ $v = scalar ]; then export SV_LIB_PATH=$(pwd)/spine-vision_amd/libsv_kernels_dwscalar.so; else unset SV_LIB_PATH; fi
  timeout -k 10 300 python tools/dw_bench.py > "$OUT/dw_$v.txt" 2>&1
  rc=$?; echo "dw $v rc=$rc"; grep -v amdgpu "$OUT/dw_$v.txt"; [ $rc -ne 0 ] && exit $rc
done
for r in 1 2; do
  for v in pk scalar; do
    if [ $v = scalar ]; then export SV_LIB_PATH=$(pwd)/spine-vision_amd/libsv_kernels_dwscalar.so; else unset SV_LIB_PATH; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_${v}_$r.json" 2> "$OUT/bench_${v}_$r.err"
    rc=$?; echo "bench $v $r rc=$rc $(python3 -c "import json; d=json.load(open('$OUT/bench_${v}_$r.json')); print(d['value'], d['ms_per_step'])" 2>/dev/null)"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
