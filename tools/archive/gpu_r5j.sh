#!/bin/bash
# round 3, session 3: AdamW with two float4 groups in flight per thread (tests, interleaved A/B against the
# previous optim.hip through the bench's adamw probe), then the secondary config lines and the loader-fed trainer
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r5j}
mkdir -p "$OUT"
ALT=$(pwd)/spine-vision_amd/libsv_kernels_optimold.so
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_trainer_gpu.py -x -q --timeout 120 --timeout-method thread -k "adamw or clip or graph" > "$OUT/tests.log" 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $OUT/tests.log)"; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" "$OUT/tests.log" | head -20; exit $rc; }
for r in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export SV_LIB_PATH=$ALT; else unset SV_LIB_PATH; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_${v}_$r.json" 2> "$OUT/bench_${v}_$r.err"
    rc=$?; echo "bench $v $r rc=$rc $(python3 -c "import json; d=json.load(open('$OUT/bench_${v}_$r.json')); k=d['roofline']['kernels']['adamw']; print(d['value'], d['ms_per_step'], 'adamw', k['avg_launch_us'], k['hbm_gbs'])" 2>/dev/null)"
    [ $rc -ne 0 ] && exit $rc
  done
done
unset SV_LIB_PATH
bash tools/gpu_configs.sh "${1:-r5j}/cfg" || exit $?
timeout -k 10 600 python bench.py --trainer --steps 30 --warmup 2 > "$OUT/trainer_device.json" 2> "$OUT/trainer_device.err"
rc=$?; echo "trainer rc=$rc $(head -c 300 $OUT/trainer_device.json)"
exit $rc
