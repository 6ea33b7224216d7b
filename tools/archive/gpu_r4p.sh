#!/bin/bash
# round 3: the classification heads as one GEMM (SV_FUSED_HEADS): classifier / trainer / golden tests,
# interleaved classification A/B, kernel trace of the fused form
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r4p}
mkdir -p "$OUT"
ROOTDIR=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_golden_r2_gpu.py tests/test_trainer_gpu.py tests/test_resnet_parity_256_gpu.py tests/test_parity_geometry_gpu.py -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $OUT/tests.log)"; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" "$OUT/tests.log" | head -20; exit $rc; }
for r in 1 2; do
  for v in 1 0; do
    SV_FUSED_HEADS=$v timeout -k 10 300 python bench.py --workload classification --steps 30 --warmup 5 --no-cpu-baseline > "$OUT/cls_${v}_$r.json" 2> "$OUT/cls_${v}_$r.err"
    rc=$?; echo "fused=$v $r rc=$rc $(python -c "import json;d=json.load(open('$OUT/cls_${v}_$r.json'));print(d['value'], d['ms_per_step'])" 2>/dev/null)"; [ $rc -ne 0 ] && exit $rc
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOTDIR/$OUT/prof" -o run -- python3 "$ROOTDIR/bench.py" --workload classification --steps 3 --warmup 3 --no-cpu-baseline > "$ROOTDIR/$OUT/prof.json" 2> "$ROOTDIR/$OUT/prof.err"
rc=$?; echo "rocprof rc=$rc"
exit $rc
