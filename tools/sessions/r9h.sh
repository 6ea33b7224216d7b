#!/bin/bash
# round 4: stride-2 dgrad straight into dx (mode 5 remapped rows, fused BN statistics) -- tests, then
# classification A/B against the slab + scatter form (SV_S2_DIRECT=0), then a kernel-trace profile
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r9h}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_resnet_gpu.py tests/test_resnet_parity_256_gpu.py tests/test_kernels_gpu.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for v in 1 0; do
    SV_S2_DIRECT=$v timeout -k 10 300 python bench.py --workload classification --steps 50 --warmup 10 --no-cpu-baseline > $O/cls_${v}_$i.json 2>>$O/bench.err || exit $?
    python -c "import json; d=json.loads(open('$O/cls_${v}_$i.json').read().strip().splitlines()[-1]); print('direct=$v', d['value'], d['ms_per_step'])"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python $GRAFT_REPO_ROOT/bench.py --workload classification --steps 20 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit $?
echo prof ok
