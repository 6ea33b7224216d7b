#!/bin/bash
# round 3: GEMM K-loop vs epilogue (no-store diagnostic build), in-kernel clock, ConvNeXt side-cap and
# comm-reserve A/B (interleaved bench runs)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r4d}
mkdir -p "$OUT"
CASES="fc1_fwd(dual),fc1_fwd(store),fc2_fwd(res),fc2_dgrad(mul),fc1_dgrad,fc2_wgrad+bias,fc1_wgrad,torch_fc1_dgrad"
timeout -k 10 300 python tools/gemm_bench.py --stages S1,S2,S3,S4,BIG --iters 10 --cases "$CASES" > "$OUT/gemm.txt" 2>&1
rc=$?; echo "gemm rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/gemm.txt"; exit $rc; }
SV_LIB_PATH=spine-vision_amd/libsv_kernels_nostore.so timeout -k 10 300 python tools/gemm_bench.py --stages S1,S2,S3,S4,BIG --iters 10 --cases "$CASES" > "$OUT/gemm_nostore.txt" 2>&1
rc=$?; echo "gemm nostore rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/gemm_nostore.txt"; exit $rc; }
timeout -k 10 120 python tools/clock_stamp.py > "$OUT/clock.txt" 2>&1
rc=$?; echo "clock rc=$rc $(tail -1 $OUT/clock.txt | head -c 600)"; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in base cap240 cap224 res16 res32; do
    case $v in
      base) E="" ;; cap240) E="SV_SIDE_GRID_CAP=240" ;; cap224) E="SV_SIDE_GRID_CAP=224" ;;
      res16) E="SV_BENCH_RESERVE=16" ;; res32) E="SV_BENCH_RESERVE=32" ;;
    esac
    env $E SV_BENCH_PROBE=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/b_${v}_$r.json" 2>"$OUT/b_${v}_$r.err"
    rc=$?; echo "$v $r rc=$rc $(python -c "import json;d=json.load(open('$OUT/b_${v}_$r.json'));print(d['value'])" 2>/dev/null)"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
