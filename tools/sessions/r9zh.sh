#!/bin/bash
# round 4: opt-in bf16 split-K slabs for the weight gradients (SV_WGRAD_BF16_SLABS) -- kernel tests, the B=32
# ConvNeXt parity test with them on, then the step A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r9zh}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_family_gpu.py > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -ne 0 ] && exit $rc
SV_WGRAD_BF16_SLABS=1 timeout -k 10 600 python -u -m pytest -x -q -s --timeout 400 --timeout-method thread tests/test_bs32_parity_gpu.py > $O/bs32.log 2>&1
echo "bs32 parity with bf16 slabs rc=$?"; grep -iE "rel|worst|median|passed|failed" $O/bs32.log | tail -8
for i in 1 2 3; do
  for v in 0 1; do
    SV_WGRAD_BF16_SLABS=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_${v}_$i.json 2>>$O/bench.err || exit $?
    python -c "import json; d=json.loads(open('$O/b_${v}_$i.json').read().strip().splitlines()[-1]); print('bf16slabs=$v', d['value'], d['ms_per_step'])"
  done
done
