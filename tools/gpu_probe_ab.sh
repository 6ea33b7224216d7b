#!/bin/bash
# cost of bench.py's live GEMM-class HIP events: interleaved runs with the probe on / off
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-probe}
mkdir -p "$OUT"
for rep in 1 2; do
  for p in 1 0; do
    SV_BENCH_PROBE=$p timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/p${p}_$rep.json" 2> "$OUT/p${p}_$rep.err"
    rc=$?; echo "probe=$p rep=$rep rc=$rc $(python -c "import json;print(json.load(open('$OUT/p${p}_$rep.json'))['value'])")"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
