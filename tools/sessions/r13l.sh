#!/bin/bash
# round 6: matrix-core depthwise -- parity of all three passes (the weight gradient is new), standalone timing with 32
# and 16 channels per workgroup (SV_DW_MFMA_CG), the training line for both, interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOTDIR=$(pwd)
N=${1:-r13l}
O=$ROOTDIR/gpurun_out/$N
mkdir -p $O
for cg in 16 32; do
  SV_DW_MFMA_CG=$cg timeout -k 10 300 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_dw_mfma_gpu.py > $O/dwm_$cg.log 2>&1 || { grep -E "FAIL|Error|assert|wgrad" $O/dwm_$cg.log | head -30; tail -20 $O/dwm_$cg.log; exit 1; }
  echo "cg $cg: $(grep -E '[0-9]+ passed|failed' $O/dwm_$cg.log)"
  SV_DW_MFMA_CG=$cg timeout -k 10 300 python -u tools/dw_bench.py --iters 20 > $O/dw_bench_$cg.txt 2>&1 || { tail -20 $O/dw_bench_$cg.txt; exit 1; }
done
grep -E "wgrad" $O/dwm_16.log | tail -12
paste <(grep -E "mfma|one-pass|wgrad|LN" $O/dw_bench_16.txt) <(grep -E "mfma|one-pass|wgrad|LN" $O/dw_bench_32.txt | awk '{print $(NF-3), $(NF-2)}')
for t in 16 32 16 32; do
  SV_DW_MFMA_CG=$t timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$t.json 2> $O/bench_$t.err || { tail -5 $O/bench_$t.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_$t.json').read().strip().splitlines()[-1]); k=d['roofline']['kernels']; print('cg $t train', d['value'], d['ms_per_step'], d['main_queue']['busy_ms_per_step'], {n: k[n]['ms_per_step'] for n in ('dw_fwd', 'dw_bwd_data', 'dw_wgrad')})"
done
