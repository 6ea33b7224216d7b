#!/bin/bash
# round 3 (late): gathered-conv LDS ring depth A/B — S = 3 (fprop / dgrad) and 4 (wgrads) against S = 6
# (144 KiB, one workgroup per CU, five tiles in flight) via SV_CONV_S / SV_WGRAD_S: conv parity tests at S = 6,
# standalone conv pass timings and the classification step, interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r6b}
mkdir -p "$OUT"
SV_CONV_S=6 SV_WGRAD_S=6 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_resnet_gpu.py tests/test_resnet_parity_256_gpu.py > "$OUT/tests_s6.txt" 2>&1
rc=$?; echo "tests S6 rc=$rc $(tail -1 $OUT/tests_s6.txt)"; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for cfg in "3 4" "6 4" "3 6" "6 6"; do
    set -- $cfg
    SV_CONV_S=$1 SV_WGRAD_S=$2 timeout -k 10 300 python tools/conv_bench.py --iters 20 > "$OUT/conv_${1}_${2}_$r.txt" 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "conv_bench $cfg rc=$rc"; exit $rc; }
  done
done
for r in 1 2; do
  for cfg in "3 4" "6 6"; do
    set -- $cfg
    SV_CONV_S=$1 SV_WGRAD_S=$2 timeout -k 10 300 python bench.py --workload classification --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_${1}_${2}_$r.json" 2> "$OUT/bench_${1}_${2}_$r.err"
    rc=$?; echo "bench $cfg r$r rc=$rc $(head -c 200 $OUT/bench_${1}_${2}_$r.json | grep -o '"value": [0-9.]*')"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
