#!/bin/bash
# Backward-GEMM A/B: standalone dgrad/wgrad timings per implementation, then the full step with the
# wgrad side stream on/off and with v8 forced (each variant one bench line)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-bab}
mkdir -p "$OUT"
IMPLS="${IMPLS:-8}" GB_ARGS="--cases dgrad,wgrad" bash tools/gpu_gemm_ab.sh "$(basename $OUT)_gemm" || exit $?
for v in ${BENCH_VARIANTS:-SV_SIDE_STREAM=1 SV_SIDE_STREAM=0 SV_SIDE_STREAM=0,SV_GEMM_IMPL=8}; do
  envs=$(echo "$v" | tr ',' ' ')
  env $envs timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.err"
  rc=$?; echo "$v bench rc=$rc $(head -c 160 "$OUT/bench_$v.json" | sed 's/.*"value": \([0-9.]*\).*/\1/')"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
