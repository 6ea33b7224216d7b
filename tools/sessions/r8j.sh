#!/bin/bash
# round 4: the spread in-kernel split-K fold -- bitwise tests (incl. uneven load), then the ConvNeXt step A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r8j}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gemm_family_gpu.py -k "fold" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for f in 1 0; do
    SV_INKERNEL_FOLD=$f timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/fold${f}_$i.json 2>>$O/bench.err || exit $?
    python -c "import json; d=json.loads(open('$O/fold${f}_$i.json').read().strip().splitlines()[-1]); k=d['roofline']['kernels']; print('fold $f', d['value'], d['ms_per_step'], 'fold_ms', k['fold']['ms_per_step'], 'wgrad_us', k['wgrad']['avg_launch_us'])"
  done
done
