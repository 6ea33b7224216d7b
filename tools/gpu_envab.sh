#!/bin/bash
# interleaved step A/B over environment settings: ENVS="A=1 B=2|A=0" (alternatives separated by |)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-envab}
mkdir -p "$OUT"
IFS='|' read -ra ALTS <<< "${ENVS}"
for rnd in 1 2; do
  i=0
  for alt in "${ALTS[@]}"; do
    env $alt timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/b_${i}_$rnd.json" 2> "$OUT/b_${i}_$rnd.err"
    rc=$?; echo "[$alt] rnd=$rnd rc=$rc $(python3 -c "import json; d=json.load(open('$OUT/b_${i}_$rnd.json')); print(d['value'], d['ms_per_step'])" 2>&1 | tail -1)"
    [ $rc -ne 0 ] && { tail -5 "$OUT/b_${i}_$rnd.err"; exit $rc; }
    i=$((i+1))
  done
done
exit 0
