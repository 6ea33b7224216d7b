#!/bin/bash
# host-lookahead A/B (SV_MAX_INFLIGHT), interleaved on one box: img/s and reserved HBM per setting
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-inflight}
mkdir -p "$OUT"
for rep in 1 2; do
  for m in ${SETTINGS:-0 2 3}; do
    SV_MAX_INFLIGHT=$m timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/m${m}_$rep.json" 2> "$OUT/m${m}_$rep.err"
    rc=$?; echo "max_inflight=$m rep=$rep rc=$rc $(python -c "import json;b=json.load(open('$OUT/m${m}_$rep.json'));print(b['value'], b.get('hbm_reserved_gb'))")"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
