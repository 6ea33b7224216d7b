#!/bin/bash
# round 4: packed-f32 GELU epilogues in v9 (default build) vs scalar (gpk0 build): bitwise tests, standalone, step, eval
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r9z}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_family_gpu.py -k "production or bitwise_vs_dispatch" > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for v in pk sc; do
  if [ $v = sc ]; then L=$(pwd)/spine-vision_amd/libsv_kernels_gpk0.so; else L=""; fi
  SV_LIB_PATH=$L timeout -k 10 300 python tools/gemm_bench.py --stages S1,S3 --iters 10 --impls 0 --cases "fc1_fwd(dual)" > $O/g_$v.txt 2>&1 || exit $?
  echo "$v"; grep -v amdgpu.ids $O/g_$v.txt
done
for i in 1 2 3; do
  for v in pk sc; do
    if [ $v = sc ]; then L=$(pwd)/spine-vision_amd/libsv_kernels_gpk0.so; else L=""; fi
    SV_LIB_PATH=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_${v}_$i.json 2>>$O/bench.err || exit $?
    SV_LIB_PATH=$L timeout -k 10 300 python bench.py --inference --steps 10 --warmup 3 --no-cpu-baseline > $O/i_${v}_$i.json 2>>$O/bench.err || exit $?
    python -c "import json; d=json.loads(open('$O/b_${v}_$i.json').read().strip().splitlines()[-1]); e=json.loads(open('$O/i_${v}_$i.json').read().strip().splitlines()[-1]); print('$v train', d['value'], 'eval', e['value'])"
  done
done
