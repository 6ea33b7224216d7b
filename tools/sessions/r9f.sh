#!/bin/bash
# round 4: 32-bit index arithmetic in the BatchNorm / pooling passes -- BN tests, then classification vs the r9a tree
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r9f}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_resnet_gpu.py tests/test_bn_small_gpu.py tests/test_resnet_parity_256_gpu.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for v in new old; do
    if [ $v = new ]; then L=""; else L=$(pwd)/spine-vision_amd/libsv_kernels_old.so; fi
    SV_LIB_PATH=$L timeout -k 10 300 python bench.py --workload classification --steps 50 --warmup 10 --no-cpu-baseline > $O/cls_${v}_$i.json 2>>$O/bench.err || exit $?
    python -c "import json; d=json.loads(open('$O/cls_${v}_$i.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
  done
done
