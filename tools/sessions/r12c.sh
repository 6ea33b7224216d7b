#!/bin/bash
# round 5: LayerNorm statistics butterfly from the cross-lane unit (xlane_group_sum) -- its bitwise test, the LayerNorm /
# depthwise / fused-MLP kernel tests, then training step and eval forward against the ds_bpermute build
# (libsv_kernels_lnshfl.so: norm.hip with -DSV_LN_XLANE=0), interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r12c}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_dw_ln_fused_gpu.py tests/test_kernels_gpu.py tests/test_mlp_fused_gpu.py > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
for v in x s; do
  L=$([ $v = x ] && echo spine-vision_amd/libsv_kernels.so || echo spine-vision_amd/libsv_kernels_lnshfl.so)
  SV_LIB_PATH=$PWD/$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_${v}_${r}.json 2>>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_${v}_${r}.json').read().strip().splitlines()[-1]); print('train $v', d['value'], d['ms_per_step'])"
done
done
for v in x s; do
  L=$([ $v = x ] && echo spine-vision_amd/libsv_kernels.so || echo spine-vision_amd/libsv_kernels_lnshfl.so)
  SV_LIB_PATH=$PWD/$L timeout -k 10 300 python bench.py --inference --steps 20 --warmup 5 --no-cpu-baseline > $O/inf_${v}.json 2>>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/inf_${v}.json').read().strip().splitlines()[-1]); print('inf $v', d['value'], d['ms_per_step'])"
done
