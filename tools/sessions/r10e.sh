#!/bin/bash
# round 5: staggered fused MLP -- bitwise tests, standalone timing, bench train / eval, PMC of the fused kernel
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r10e}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_mlp_fused_gpu.py > $O/t_mlp.log 2>&1 || { tail -40 $O/t_mlp.log; exit 1; }
grep -cE "PASSED" $O/t_mlp.log
timeout -k 10 300 python tools/mlp_bench.py --shapes base-S1,base-S2,large-S1 > $O/mlp_bench.txt 2>&1 || { tail -20 $O/mlp_bench.txt; exit 1; }
cat $O/mlp_bench.txt
for v in on off; do
  E=$([ $v = on ] && echo SV_FUSED_MLP=1 || echo SV_FUSED_MLP=0)
  env $E timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_$v.json 2>>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
  env $E timeout -k 10 300 python bench.py --inference --steps 20 --warmup 5 --no-cpu-baseline > $O/inf_$v.json 2>>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]); e=json.loads(open('$O/inf_$v.json').read().strip().splitlines()[-1]); print('$v train', d['value'], d['ms_per_step'], 'eval', e['value'])"
done
PMC_SETS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_WR
GRBM_GUI_ACTIVE GRBM_COUNT" CMD="tools/mlp_bench.py --shapes base-S1 --iters 3" bash tools/pmc_run.sh ${1:-r10e}/pmc || exit 1
python tools/pmc_dump.py $O/pmc mlp_fwd gemm9 > $O/pmc.txt
grep -E "==|split|busy" $O/pmc.txt
