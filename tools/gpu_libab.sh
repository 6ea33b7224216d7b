#!/bin/bash
# A/B of prebuilt library variants (SV_LIB_PATH): standalone depthwise timings, then interleaved steps
# LIBS="a.so b.so" bash tools/gpu_libab.sh OUT
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-libab}
mkdir -p "$OUT"
for l in $LIBS; do
  SV_LIB_PATH=$(pwd)/$l timeout -k 10 300 python tools/dw_bench.py ${DWARGS:-} > "$OUT/dw_$(basename $l).txt" 2>&1
  rc=$?; echo "== $l rc=$rc"; grep -v amdgpu "$OUT/dw_$(basename $l).txt"
  [ $rc -ne 0 ] && exit $rc
done
ENVS=$(for l in $LIBS; do printf "SV_LIB_PATH=%s|" "$(pwd)/$l"; done)
ENVS="${ENVS%|}" bash tools/gpu_envab.sh "${1:-libab}/ab"
