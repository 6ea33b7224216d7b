#!/bin/bash
# round 5: fused MLP correctness, the ConvNeXt bf16 emulation parity (B=2 geometry, base B=32, large B=64), the advisor
# fixes, then the bench with the fused MLP on / off (training and eval forward)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r10b}
mkdir -p $O
T="python -u -m pytest -x -v -s --timeout 900 --timeout-method thread"
timeout -k 10 600 $T tests/test_mlp_fused_gpu.py "tests/test_gemm_family_gpu.py::test_wgrad_inkernel_fold_bitwise" > $O/t_mlp.log 2>&1 || { tail -40 $O/t_mlp.log; exit 1; }
grep -E "PASSED|FAILED" $O/t_mlp.log | tail -40
for v in on off; do
  E=$([ $v = on ] && echo SV_FUSED_MLP=1 || echo SV_FUSED_MLP=0)
  env $E timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_$v.json 2>>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
  env $E timeout -k 10 300 python bench.py --inference --steps 20 --warmup 5 --no-cpu-baseline > $O/inf_$v.json 2>>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]); e=json.loads(open('$O/inf_$v.json').read().strip().splitlines()[-1]); print('$v train', d['value'], d['ms_per_step'], 'eval', e['value'])"
done
timeout -k 10 1500 $T tests/test_parity_geometry_gpu.py tests/test_bs32_parity_gpu.py tests/test_resnet_parity_256_gpu.py tests/test_comm_reserve_gpu.py > $O/t_parity.log 2>&1 || { grep -E "\[parity\]|\[emu\]|PASS|FAIL|Error" $O/t_parity.log | tail -40; exit 1; }
grep -E "\[parity\]|\[comm\]|PASSED|FAILED" $O/t_parity.log | tail -60
cp gpurun_out/comm_latency.json $O/ 2>/dev/null; true
