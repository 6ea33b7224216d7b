#!/bin/bash
# round 4: classification A/B, gathered forward split threshold 64 (new default) vs 32 (round 3)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r8f}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_resnet_gpu.py -k "split or bn_stats or fwd" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for k in 64 32; do
    SV_CONV_FWD_MIN_KSTEPS=$k timeout -k 10 300 python bench.py --workload classification --steps 50 --warmup 10 --no-cpu-baseline > $O/cls_k${k}_$i.json 2>>$O/bench.err || exit $?
    python -c "import json; d=json.loads(open('$O/cls_k${k}_$i.json').read().strip().splitlines()[-1]); print('minks $k', d['value'], d['ms_per_step'])"
  done
done
