#!/bin/bash
# round 5: fused MLP backward at C = 128 -- tests, standalone timing against the three kernels, bench on / off
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r10k}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_mlp_fused_gpu.py ${MLPK:+-k "$MLPK"} > $O/t_mlp.log 2>&1 || { grep -E "FAIL|Error|assert" $O/t_mlp.log | head -20; tail -30 $O/t_mlp.log; exit 1; }
grep -cE "PASSED" $O/t_mlp.log; grep "fused bwd" $O/t_mlp.log
timeout -k 10 300 python tools/mlp_bench.py --shapes base-S1 --bwd > $O/mlp_bench.txt 2>&1 || { tail -20 $O/mlp_bench.txt; exit 1; }
cat $O/mlp_bench.txt
for v in on off; do
  E=$([ $v = on ] && echo SV_FUSED_MLP_BWD=1 || echo SV_FUSED_MLP_BWD=0)
  env $E timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_$v.json 2>>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]); print('$v train', d['value'], d['ms_per_step'])"
done
[ -n "${SKIP_PARITY:-}" ] && exit 0
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread tests/test_bs32_parity_gpu.py::test_convnext_base_512_bs32_bf16_step "tests/test_parity_geometry_gpu.py::test_convnext_bf16_geometry" tests/test_parity_geometry_gpu.py::test_convnext_bf16_schedule_knobs_match_default > $O/t_parity.log 2>&1 || { grep -E "\[parity\]|FAIL|Error" $O/t_parity.log | tail -20; exit 1; }
grep -E "\[parity\]|PASSED" $O/t_parity.log
