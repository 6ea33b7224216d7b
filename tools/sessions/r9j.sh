#!/bin/bash
# round 4: stride-2 dgrads straight into dx incl. the 1x1 shortcut's accumulate (class (0, 0) alone) --
# ResNet tests, then classification: b = default, d = no split-K for the strided dgrads (SV_S2_NOSPLIT),
# o = slabs + scatter (SV_S2_DIRECT=0)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r9j}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_resnet_gpu.py tests/test_resnet_parity_256_gpu.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for v in b d o; do
    case $v in b) E="SV_S2_NOSPLIT=0";; d) E="SV_S2_NOSPLIT=1";; o) E="SV_S2_DIRECT=0";; esac
    env $E timeout -k 10 300 python bench.py --workload classification --steps 50 --warmup 10 --no-cpu-baseline > $O/cls_${v}_$i.json 2>>$O/bench.err || exit $?
    python -c "import json; d=json.loads(open('$O/cls_${v}_$i.json').read().strip().splitlines()[-1]); print('$v $E', d['value'], d['ms_per_step'])"
  done
done
