#!/bin/bash
# round 6: the matrix-core depthwise conv with the buffer-load fill (wave = input rows, descriptor range check for
# the image border): parity, standalone timing, the training line on / off, then the whole GPU suite with it ON
# (SV_DW_MFMA=1: the emulation rounds the depthwise operands to bf16 the same way)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOTDIR=$(pwd)
N=${1:-r13g}
O=$ROOTDIR/gpurun_out/$N
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_dw_mfma_gpu.py > $O/dwm.log 2>&1 || { grep -E "FAIL|Error|assert|dw mfma" $O/dwm.log | head -40; tail -30 $O/dwm.log; exit 1; }
grep -E "passed|failed" $O/dwm.log
timeout -k 10 300 python -u tools/dw_bench.py --iters 20 > $O/dw_bench.txt 2>&1 || { tail -20 $O/dw_bench.txt; exit 1; }
grep -E "bf16dz acc|LN" $O/dw_bench.txt
run_bench() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$tag.json 2> $O/bench_$tag.err || { tail -5 $O/bench_$tag.err; return 1; }
  python -c "import json; d=json.loads(open('$O/bench_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['value'], d['ms_per_step'], d['main_queue']['busy_ms_per_step'])"
}
run_bench dwmfma SV_DW_MFMA=1 && run_bench valu SV_DW_MFMA=0 && run_bench dwmfma2 SV_DW_MFMA=1 || exit 1
SV_DW_MFMA=1 timeout -k 10 900 python -u -m pytest --maxfail=8 -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1
echo "suite exit $?"; grep -E "^FAILED|passed|failed" $O/tests.log | tail -12
