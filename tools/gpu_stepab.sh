#!/bin/bash
# step-level A/B of kernel choices (one bench line per variant, same box, interleaved order)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-stepab}
mkdir -p "$OUT"
i=0
for v in ${VARIANTS:-"BASE=1"}; do
  i=$((i+1))
  envs=$(echo "$v" | tr ',' ' ')
  env $envs timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/v$i.json" 2> "$OUT/v$i.err"
  rc=$?
  val=$(python -c "import json;d=json.load(open('$OUT/v$i.json'));print(d['value'], d['ms_per_step'])" 2>/dev/null)
  echo "$v rc=$rc $val" | tee -a "$OUT/summary.txt"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
