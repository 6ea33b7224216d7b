#!/bin/bash
# round 5: the fused S1 MLP backward with cross-lane butterflies and a full vmcnt drain before the LayerNorm operands
# (SV_XLANE in mlp.hip) -- its tests (run-to-run equality included) twice, two localization digests against the previous
# build (libsv_kernels_prev.so), then the training step A/B interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r12g}
mkdir -p $O
PREV=$PWD/spine-vision_amd/libsv_kernels_prev.so
for k in 1 2; do
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_mlp_fused_gpu.py > $O/tests_$k.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests_$k.log | head -20; tail -5 $O/tests_$k.log; exit 1; }
tail -1 $O/tests_$k.log
done
timeout -k 10 300 python tools/step_digest.py --workload localization > $O/d1.json 2>> $O/d.err && timeout -k 10 300 python tools/step_digest.py --workload localization > $O/d2.json 2>> $O/d.err && SV_LIB_PATH=$PREV timeout -k 10 300 python tools/step_digest.py --workload localization > $O/d3.json 2>> $O/d.err || { tail -20 $O/d.err; exit 1; }
cat $O/d1.json $O/d2.json $O/d3.json
for r in 1 2 3; do
for v in n p; do
  L=$([ $v = n ] && echo $PWD/spine-vision_amd/libsv_kernels.so || echo $PREV)
  SV_LIB_PATH=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_${v}_${r}.json 2>>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_${v}_${r}.json').read().strip().splitlines()[-1]); print('train $v', d['value'], d['ms_per_step'])"
done
done
