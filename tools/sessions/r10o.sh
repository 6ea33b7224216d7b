#!/bin/bash
# round 5: fused MLP forward at C = 512 (S3) -- tests, standalone timing against the two GEMMs, bench train / eval A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r10o}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_mlp_fused_gpu.py -k "not bwd" > $O/t_mlp.log 2>&1 || { grep -E "FAIL|Error|assert" $O/t_mlp.log | head -20; tail -30 $O/t_mlp.log; exit 1; }
grep -cE "PASSED" $O/t_mlp.log
timeout -k 10 300 python tools/mlp_bench.py --shapes base-S3,base-S2 > $O/mlp_bench.txt 2>&1 || { tail -20 $O/mlp_bench.txt; exit 1; }
cat $O/mlp_bench.txt
[ -n "${SKIP_BENCH:-}" ] && exit 0
for v in on off; do
  E=$([ $v = on ] && echo SV_FUSED_MLP_C=128,192,256,512 || echo SV_FUSED_MLP_C=128,192,256)
  env $E timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_$v.json 2>>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
  env $E timeout -k 10 300 python bench.py --inference --steps 20 --warmup 5 --no-cpu-baseline > $O/i_$v.json 2>>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]); e=json.loads(open('$O/i_$v.json').read().strip().splitlines()[-1]); print('$v train', d['value'], d['ms_per_step'], 'eval', e['value'], e['ms_per_step'])"
done
