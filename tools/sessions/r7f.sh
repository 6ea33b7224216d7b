#!/bin/bash
# round 4: step A/B of the in-kernel fold variants and the depthwise XCD order (interleaved, 20 steps each)
set -u
O=gpurun_out/r7f
mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/$n.json 2>>$O/bench.err || exit $?
  python -c "import json; d=json.load(open('$O/$n.json')); k=d['roofline']['kernels']; print('$n', d['value'], d['ms_per_step'], 'fold', k.get('fold',{}).get('ms_per_step'), 'dw_wgrad', k.get('dw_wgrad',{}).get('us_per_launch'))"
}
for i in 1 2; do
  run base_$i SV_INKERNEL_FOLD=0
  run dwxcd0_$i SV_INKERNEL_FOLD=0 SV_DW_XCD=0
  run fold_s4_$i SV_FOLD_MAX_SPLIT=4
  run fold_wgs128_$i SV_WGRAD9_WGS=128 SV_FOLD_MAX_SPLIT=8
  run nofold_wgs128_$i SV_INKERNEL_FOLD=0 SV_WGRAD9_WGS=128
done
