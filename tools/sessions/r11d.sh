#!/bin/bash
# round 5: BatchNorm statistics folds (in-pass fold kernels, chunk-split finishes) -- bitwise tests, ResNet tests,
# classification A/B of the split finish
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
N=${1:-r11d}
O=gpurun_out/$N
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_bn_fold_gpu.py > $O/t_fold.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" $O/t_fold.log | head -30; tail -30 $O/t_fold.log; exit 1; }
grep -c PASSED $O/t_fold.log
[ -n "${FOLD_ONLY:-}" ] && exit 0
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_resnet_gpu.py tests/test_bn_small_gpu.py > $O/t_resnet.log 2>&1 || { grep -E "FAIL|Error|assert" $O/t_resnet.log | head -30; tail -30 $O/t_resnet.log; exit 1; }
grep -c PASSED $O/t_resnet.log
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_resnet_parity_256_gpu.py tests/test_bs32_parity_gpu.py::test_resnet50_256_bs32_bf16_step tests/test_parity_geometry_gpu.py::test_resnet_bf16_side_stream_matches_single_stream tests/test_trainer_gpu.py > $O/t_parity.log 2>&1 || { grep -E "\[parity\]|FAIL|Error|assert" $O/t_parity.log | tail -30; exit 1; }
grep -E "\[parity\]" $O/t_parity.log | tail -30; grep -c PASSED $O/t_parity.log
for r in 1 2; do
for v in 1 0; do
  SV_FIN_SPLIT=$v timeout -k 10 300 python bench.py --workload classification --steps 30 --warmup 5 --no-cpu-baseline > $O/b_fold${v}_$r.json 2>>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_fold${v}_$r.json').read().strip().splitlines()[-1]); print('split=$v', d['value'], d['ms_per_step'])"
done
done
