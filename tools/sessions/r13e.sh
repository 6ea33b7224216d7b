#!/bin/bash
# round 6: first run of the matrix-core depthwise conv (csrc/dwmfma.hip): its parity test, the standalone timing
# beside the VALU kernels, then the training line with SV_DW_MFMA=1 against the default
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOTDIR=$(pwd)
N=${1:-r13e}
O=$ROOTDIR/gpurun_out/$N
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_dw_mfma_gpu.py > $O/dwm.log 2>&1 || { grep -E "FAIL|Error|assert|dw mfma" $O/dwm.log | head -40; tail -30 $O/dwm.log; exit 1; }
grep -E "dw mfma|passed|failed" $O/dwm.log
timeout -k 10 300 python -u tools/dw_bench.py --iters 20 > $O/dw_bench.txt 2>&1 || { tail -20 $O/dw_bench.txt; exit 1; }
cat $O/dw_bench.txt
for f in 1 0; do
  SV_DW_MFMA=$f timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$f.json 2> $O/bench_$f.err || { tail -5 $O/bench_$f.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_$f.json').read().strip().splitlines()[-1]); print('dw_mfma=$f train', d['value'], d['ms_per_step'], d.get('main_queue'))"
done
