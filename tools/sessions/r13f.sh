#!/bin/bash
# round 6: the matrix-core depthwise conv (csrc/dwmfma.hip) parity + standalone timing, the fused fc1 dgrad + LN
# backward test, the training line A/Bs (fusion on / off, matrix-core depthwise on), then the whole GPU suite
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOTDIR=$(pwd)
N=${1:-r13f}
O=$ROOTDIR/gpurun_out/$N
mkdir -p $O
timeout -k 10 300 python -u -m pytest -v -s --timeout 200 --timeout-method thread tests/test_dw_mfma_gpu.py > $O/dwm.log 2>&1
echo "dw mfma test exit $?"; grep -E "dw mfma|passed|failed|Error" $O/dwm.log | head -40
timeout -k 10 300 python -u tools/dw_bench.py --iters 20 > $O/dw_bench.txt 2>&1 || { tail -20 $O/dw_bench.txt; exit 1; }
cat $O/dw_bench.txt
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_ln_bwd_fused_gpu.py > $O/ln.log 2>&1 || { grep -E "FAIL|Error|assert|ln_bwd fused" $O/ln.log | head -30; tail -30 $O/ln.log; exit 1; }
grep -E "passed|failed" $O/ln.log
run_bench() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$tag.json 2> $O/bench_$tag.err || { tail -5 $O/bench_$tag.err; return 1; }
  python -c "import json; d=json.loads(open('$O/bench_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['value'], d['ms_per_step'], d.get('main_queue'))"
}
run_bench default SV_FUSED_LN_BWD=1 && run_bench noln SV_FUSED_LN_BWD=0 && run_bench dwmfma SV_DW_MFMA=1 || exit 1
timeout -k 10 900 python -u -m pytest --maxfail=5 -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
