#!/bin/bash
# round 3, session 3: v9 epilogue with 8-row x 128-B bf16 accesses (family / parity tests, standalone A/B
# against the 16 x 64-B build, interleaved bench lines) and the per-CU store rate
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r5c}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gemm_family_gpu.py tests/test_kernels_gpu.py tests/test_backbone_gpu.py tests/test_resnet_gpu.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $OUT/tests.log)"; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" "$OUT/tests.log" | head -20; exit $rc; }
timeout -k 10 120 ./tools/store_shape > "$OUT/store_shape.txt" 2>&1
rc=$?; echo "store_shape rc=$rc"; tail -4 "$OUT/store_shape.txt"; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in r128 r64; do
    if [ $v = r64 ]; then export SV_LIB_PATH=$(pwd)/spine-vision_amd/libsv_kernels_r64.so; else unset SV_LIB_PATH; fi
    timeout -k 10 300 python tools/gemm_bench.py --cases "fc1_fwd(dual),fc1_fwd(store),fc2_dgrad(mul),fc1_dgrad" --stages S1,S2,S3,S4 > "$OUT/gemm_${v}_$r.txt" 2>&1
    rc=$?; echo "gemm $v $r rc=$rc"; grep -v amdgpu "$OUT/gemm_${v}_$r.txt"; [ $rc -ne 0 ] && exit $rc
  done
done
for r in 1 2; do
  for v in r128 r64; do
    if [ $v = r64 ]; then export SV_LIB_PATH=$(pwd)/spine-vision_amd/libsv_kernels_r64.so; else unset SV_LIB_PATH; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_${v}_$r.json" 2> "$OUT/bench_${v}_$r.err"
    rc=$?; echo "bench $v $r rc=$rc $(python3 -c "import json; d=json.load(open('$OUT/bench_${v}_$r.json')); print(d['value'], d['ms_per_step'])" 2>/dev/null)"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
