#!/bin/bash
# round 5: the fused multi-task classification loss -- tests, classification A/B (SV_FUSED_LOSS), queue breakdown
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOTDIR=$(pwd)
N=${1:-r11j}
O=$ROOTDIR/gpurun_out/$N
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_head_loss_gpu.py tests/test_trainer_gpu.py "tests/test_resnet_gpu.py::test_classifier_logits_match_reference" tests/test_golden_r2_gpu.py > $O/t.log 2>&1 || { grep -E "FAIL|Error|assert" $O/t.log | head -30; tail -30 $O/t.log; exit 1; }
grep -c PASSED $O/t.log
for r in 1 2 3; do
for v in 0 1; do
  SV_FUSED_LOSS=$v timeout -k 10 300 python bench.py --workload classification --steps 40 --warmup 8 --no-cpu-baseline > $O/b_loss${v}_$r.json 2>>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_loss${v}_$r.json').read().strip().splitlines()[-1]); print('fused_loss=$v', d['value'], d['ms_per_step'])"
done
done
