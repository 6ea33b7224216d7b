#!/bin/bash
# round 6: matrix-core depthwise with the paired-column plane fill (one dword per channel and column pair, DPP swap):
# parity, standalone timing, ConvNeXt parity tests, the training line twice
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOTDIR=$(pwd)
N=${1:-r13y}
O=$ROOTDIR/gpurun_out/$N
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_dw_mfma_gpu.py > $O/dwm.log 2>&1 || { grep -E "FAIL|Error|assert" $O/dwm.log | head -20; tail -20 $O/dwm.log; exit 1; }
grep -E "passed|failed" $O/dwm.log
timeout -k 10 300 python -u tools/dw_bench.py --iters 20 > $O/dw_bench.txt 2>&1 || { tail -20 $O/dw_bench.txt; exit 1; }
grep -E "mfma fwd|mfma bwd" $O/dw_bench.txt
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_parity_geometry_gpu.py tests/test_bs32_parity_gpu.py -k "convnext" > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | head -20; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$i.json 2> $O/bench_$i.err || { tail -5 $O/bench_$i.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_$i.json').read().strip().splitlines()[-1]); k=d['roofline']['kernels']; print('train', d['value'], d['ms_per_step'], d['main_queue']['busy_ms_per_step'], {n: k[n]['ms_per_step'] for n in ('dw_fwd', 'dw_bwd_data')})"
done
