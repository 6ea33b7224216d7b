#!/bin/bash
# round 6: the matrix-core depthwise weight gradient (dw7_wgrad_mfma_kernel): parity, standalone timing beside the VALU
# ring kernel, the training line with it (default) and with the VALU one (SV_DW_MFMA... the wgrad follows DW_MFMA)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOTDIR=$(pwd)
N=${1:-r13k}
O=$ROOTDIR/gpurun_out/$N
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_dw_mfma_gpu.py > $O/dwm.log 2>&1 || { grep -E "FAIL|Error|assert|wgrad" $O/dwm.log | head -40; tail -30 $O/dwm.log; exit 1; }
grep -E "wgrad|passed|failed" $O/dwm.log | tail -14
timeout -k 10 300 python -u tools/dw_bench.py --iters 20 > $O/dw_bench.txt 2>&1 || { tail -20 $O/dw_bench.txt; exit 1; }
grep -E "wgrad" $O/dw_bench.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); k=d['roofline']['kernels']; print('train', d['value'], d['ms_per_step'], d['main_queue']['busy_ms_per_step'], {n: k[n]['ms_per_step'] for n in ('dw_fwd', 'dw_bwd_data', 'dw_wgrad')})"
