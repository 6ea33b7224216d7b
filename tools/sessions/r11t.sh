#!/bin/bash
# round 5: BatchNorm activation / backward-apply passes with the channel parameters hoisted (SV_BN_FIXC) -- tests and
# classification A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r11t}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_resnet_gpu.py tests/test_bn_small_gpu.py tests/test_bn_fold_gpu.py tests/test_resnet_parity_256_gpu.py > $O/t.log 2>&1 || { grep -E "FAIL|Error|assert" $O/t.log | head -20; tail -20 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in 1 2 3; do
for v in 0 1; do
  SV_BN_FIXC=$v timeout -k 10 300 python bench.py --workload classification --steps 40 --warmup 8 --no-cpu-baseline > $O/b_${v}_${r}.json 2>>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_${v}_${r}.json').read().strip().splitlines()[-1]); print('fixc=$v', d['value'], d['ms_per_step'])"
done
done
