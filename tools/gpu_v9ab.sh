#!/bin/bash
# step-level A/B of the v9 GEMM dispatch (SV_V9: 0 off, 1 forward only, 2 everywhere; S = side stream off)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-v9ab}
mkdir -p "$OUT"
for rnd in 1 2; do
  for cfg in ${CFGS:-0 1 2 2S}; do
    mode=${cfg%S}; side=1; [ "$cfg" != "$mode" ] && side=0
    SV_V9=$mode SV_SIDE_STREAM=$side timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/b_${cfg}_$rnd.json" 2> "$OUT/b_${cfg}_$rnd.err"
    rc=$?; echo "cfg=$cfg rnd=$rnd rc=$rc $(python3 -c "import json,sys; d=json.load(open('$OUT/b_${cfg}_$rnd.json')); print(d['value'], d['ms_per_step'], d.get('loss'))" 2>&1 | tail -1)"
    [ $rc -ne 0 ] && { tail -5 "$OUT/b_${cfg}_$rnd.err"; exit $rc; }
  done
done
exit 0
