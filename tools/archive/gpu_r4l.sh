#!/bin/bash
# round 3: v9 K-loop wave priority A/B (tools/build_prio.sh libraries): standalone GEMMs, interleaved
# ConvNeXt steps and classification steps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r4l}
mkdir -p "$OUT"
LIBS="libsv_kernels.so libsv_kernels_prio1.so libsv_kernels_prio2.so"
CASES="fc1_fwd(dual),fc1_fwd(store),fc2_fwd(res),fc2_dgrad(mul),fc1_dgrad,fc2_wgrad+bias,fc1_wgrad"
for l in $LIBS; do
  SV_LIB_PATH=$(pwd)/spine-vision_amd/$l timeout -k 10 300 python tools/gemm_bench.py --stages S1,S2,S3,S4 --iters 10 --cases "$CASES" > "$OUT/gemm_$l.txt" 2>&1
  rc=$?; echo "gemm $l rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/gemm_$l.txt"; exit $rc; }
done
for r in 1 2; do
  for l in $LIBS; do
    SV_LIB_PATH=$(pwd)/spine-vision_amd/$l SV_BENCH_PROBE=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/b_${l}_$r.json" 2>"$OUT/b_${l}_$r.err"
    rc=$?; echo "$l $r rc=$rc $(python -c "import json;d=json.load(open('$OUT/b_${l}_$r.json'));print(d['value'])" 2>/dev/null)"
    [ $rc -ne 0 ] && exit $rc
  done
done
for l in $LIBS; do
  SV_LIB_PATH=$(pwd)/spine-vision_amd/$l timeout -k 10 300 python bench.py --workload classification --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/c_${l}.json" 2>"$OUT/c_${l}.err"
  rc=$?; echo "cls $l rc=$rc $(python -c "import json;d=json.load(open('$OUT/c_${l}.json'));print(d['value'])" 2>/dev/null)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
