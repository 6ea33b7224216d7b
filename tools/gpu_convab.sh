#!/bin/bash
# conv pass timings under a few split-target settings (tools/conv_bench.py), one process each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-convab}
mkdir -p "$OUT"
for cfg in ${CFGS:-""}; do
  env $cfg timeout -k 10 120 python tools/conv_bench.py >> "$OUT/conv.txt" 2>> "$OUT/conv.err" || exit $?
done
cat "$OUT/conv.txt"
