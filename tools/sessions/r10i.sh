#!/bin/bash
# round 5: the C = 128 prefetching fused MLP (y by per-wave DMA a tile ahead, x a chunk ahead) vs the general kernel
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r10i}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_mlp_fused_gpu.py > $O/t_mlp.log 2>&1 || { tail -40 $O/t_mlp.log; exit 1; }
grep -cE "PASSED" $O/t_mlp.log
timeout -k 10 300 python tools/mlp_bench.py --shapes base-S1,base-S2 > $O/mlp_bench.txt 2>&1 || { tail -20 $O/mlp_bench.txt; exit 1; }
SV_MLP128_V1=1 timeout -k 10 300 python tools/mlp_bench.py --shapes base-S1 > $O/mlp_bench_v1.txt 2>&1 || { tail -20 $O/mlp_bench_v1.txt; exit 1; }
cat $O/mlp_bench.txt $O/mlp_bench_v1.txt
for v in on off; do
  E=$([ $v = on ] && echo SV_FUSED_MLP=1 || echo SV_FUSED_MLP=0)
  env $E timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_$v.json 2>>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
  env $E timeout -k 10 300 python bench.py --inference --steps 20 --warmup 5 --no-cpu-baseline > $O/inf_$v.json 2>>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]); e=json.loads(open('$O/inf_$v.json').read().strip().splitlines()[-1]); print('$v train', d['value'], d['ms_per_step'], 'eval', e['value'])"
done
