#!/bin/bash
# round 4: one-launch BatchNorms (layers 3-4) -- bitwise tests, ResNet tests, classification A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r8b}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bn_small_gpu.py > $O/tests_small.log 2>&1
rc=$?; tail -3 $O/tests_small.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_resnet_gpu.py tests/test_resnet_parity_256_gpu.py > $O/tests_resnet.log 2>&1
rc=$?; tail -3 $O/tests_resnet.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for s in 1 0; do
    SV_BN_SMALL=$s timeout -k 10 300 python bench.py --workload classification --steps 30 --warmup 5 --no-cpu-baseline > $O/cls_small${s}_$i.json 2>>$O/bench.err || exit $?
    python -c "import json; d=json.loads(open('$O/cls_small${s}_$i.json').read().strip().splitlines()[-1]); print('small $s', d['value'], d['ms_per_step'])"
  done
done
