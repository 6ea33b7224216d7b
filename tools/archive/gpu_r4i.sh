#!/bin/bash
# depthwise wgrad grid size sweep (SV_DW_WGRAD_WGS) standalone, then in the step
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r4i}
mkdir -p "$OUT"
for w in 512 1024 2048; do
  SV_DW_WGRAD_WGS=$w timeout -k 10 200 python tools/dw_bench.py --iters 20 > "$OUT/dw_$w.txt" 2>&1
  echo "wgs $w rc=$?"; grep wgrad "$OUT/dw_$w.txt"
done
for r in 1 2; do
  for w in 512 1024 2048; do
    SV_DW_WGRAD_WGS=$w SV_BENCH_PROBE=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/b_${w}_$r.json" 2>"$OUT/b_${w}_$r.err"
    echo "bench wgs $w run $r rc=$? $(python -c "import json;print(json.load(open('$OUT/b_${w}_$r.json'))['value'])" 2>/dev/null)"
  done
done
exit 0
