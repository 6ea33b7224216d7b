#!/bin/bash
# round 5: fold kernel timing (graph-replayed) against finish + act, with diagnostic knobs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r11e}
mkdir -p $O
for cfg in "SV_FOLD_MAX_GRID=2048" "SV_FOLD_MAX_GRID=256" "SV_FOLD_MAX_GRID=256 SV_FOLD_DIAG=1" "SV_FOLD_MAX_GRID=128" "SV_FOLD_MAX_GRID=512"; do
  echo "== $cfg"
  env $cfg timeout -k 10 120 python tools/fold_bench.py > $O/fb.txt 2>&1 || { tail -20 $O/fb.txt; exit 1; }
  grep rows $O/fb.txt
done
