#!/bin/bash
# round 5: one-pass depthwise conv + LayerNorm (SV_DW_LN_FUSED) -- bitwise tests, then the training step and the eval
# forward A/B against the two launches, interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r11z}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_dw_ln_fused_gpu.py "tests/test_kernels_gpu.py::test_dwconv7_fwd_bwd" > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
grep -c PASSED $O/tests.log
for r in 1 2; do
for v in 1 0; do
  SV_DW_LN_FUSED=$v timeout -k 10 300 python bench.py --inference --steps 20 --warmup 5 --no-cpu-baseline > $O/inf_${v}_${r}.json 2>>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/inf_${v}_${r}.json').read().strip().splitlines()[-1]); print('inf fused=$v', d['value'], d['ms_per_step'])"
  SV_DW_LN_FUSED=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_${v}_${r}.json 2>>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_${v}_${r}.json').read().strip().splitlines()[-1]); print('train fused=$v', d['value'], d['ms_per_step'])"
done
done
