#!/bin/bash
# round 6: the fc1 dgrad + LayerNorm backward fusion (sv_gemm SV_EPI_LN_BWD).  Its own parity test first, then the
# whole GPU suite (the fused form is now the ConvNeXt backward's default at S3/S4), then the training line with the
# fusion on and off (SV_FUSED_LN_BWD=0) for the A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOTDIR=$(pwd)
N=${1:-r13d}
O=$ROOTDIR/gpurun_out/$N
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_ln_bwd_fused_gpu.py > $O/ln.log 2>&1 || { grep -E "FAIL|Error|assert|ln_bwd fused" $O/ln.log | head -30; tail -30 $O/ln.log; exit 1; }
grep -E "ln_bwd fused|passed|failed" $O/ln.log
timeout -k 10 900 python -u -m pytest --maxfail=5 -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for f in 1 0; do
  SV_FUSED_LN_BWD=$f timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$f.json 2> $O/bench_$f.err || { tail -5 $O/bench_$f.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_$f.json').read().strip().splitlines()[-1]); print('fused_ln=$f train', d['value'], d['ms_per_step'], d.get('main_queue'))"
done
