#!/bin/bash
# round 5: every xor butterfly from the cross-lane unit (SV_XLANE: wave_sum, LayerNorm statistics, statistics
# epilogues, the fused S1 MLP backward's LayerNorm sums) -- bitwise digests against the shuffle build
# (libsv_kernels_xoff.so: all sources with -DSV_XLANE=0), kernel tests, then the two training steps A/B, interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r12e}
mkdir -p $O
AB=$PWD/spine-vision_amd/libsv_kernels_xoff.so
for w in $DIGEST_WORKLOADS; do
  timeout -k 10 300 python tools/step_digest.py --workload $w > $O/d_${w}_1.json 2>> $O/d.err && timeout -k 10 300 python tools/step_digest.py --workload $w > $O/d_${w}_2.json 2>> $O/d.err && SV_LIB_PATH=$AB timeout -k 10 300 python tools/step_digest.py --workload $w > $O/d_${w}_ab2.json 2>> $O/d.err && SV_LIB_PATH=$AB timeout -k 10 300 python tools/step_digest.py --workload $w > $O/d_${w}_ab.json 2>> $O/d.err || { tail -20 $O/d.err; exit 1; }
  cat $O/d_${w}_1.json $O/d_${w}_2.json $O/d_${w}_ab.json $O/d_${w}_ab2.json
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_mlp_fused_gpu.py tests/test_dw_ln_fused_gpu.py tests/test_kernels_gpu.py tests/test_resnet_gpu.py tests/test_bn_small_gpu.py tests/test_bn_fold_gpu.py tests/test_head_loss_gpu.py > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
for v in x s; do
  L=$([ $v = x ] && echo $PWD/spine-vision_amd/libsv_kernels.so || echo $AB)
  SV_LIB_PATH=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_${v}_${r}.json 2>>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_${v}_${r}.json').read().strip().splitlines()[-1]); print('train $v', d['value'], d['ms_per_step'])"
done
done
for r in 1 2; do
for v in x s; do
  L=$([ $v = x ] && echo $PWD/spine-vision_amd/libsv_kernels.so || echo $AB)
  SV_LIB_PATH=$L timeout -k 10 300 python bench.py --workload classification --steps 30 --warmup 5 --no-cpu-baseline > $O/c_${v}_${r}.json 2>>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/c_${v}_${r}.json').read().strip().splitlines()[-1]); print('cls $v', d['value'], d['ms_per_step'])"
done
done
