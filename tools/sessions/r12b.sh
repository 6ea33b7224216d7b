#!/bin/bash
# round 5: the one-pass depthwise + LayerNorm in the eval forward by default -- its bitwise test and the eval / predict
# tests, then eval forward and training step at the default vs SV_DW_LN_FUSED=0, interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r12b}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_dw_ln_fused_gpu.py "tests/test_kernels_gpu.py::test_dwconv7_fwd_bwd" $EVAL_TESTS > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
for v in d 0; do
  E=$([ $v = d ] && echo SV_DW_LN_UNUSED=1 || echo SV_DW_LN_FUSED=0)
  env $E timeout -k 10 300 python bench.py --inference --steps 20 --warmup 5 --no-cpu-baseline > $O/inf_${v}_${r}.json 2>>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/inf_${v}_${r}.json').read().strip().splitlines()[-1]); print('inf mode=$v', d['value'], d['ms_per_step'])"
  env $E timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_${v}_${r}.json 2>>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_${v}_${r}.json').read().strip().splitlines()[-1]); print('train mode=$v', d['value'], d['ms_per_step'])"
done
done
