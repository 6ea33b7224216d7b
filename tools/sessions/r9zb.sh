#!/bin/bash
# round 4: ConvNeXt-large bs64 weight-gradient workgroup targets (SV_WGRAD9_WGS / SV_WGRAD9_LONG_GFLOP)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r9zb}
mkdir -p $O
for i in 1 2; do
  for v in def w192 w256 long300; do
    case $v in def) E="SV_WGRAD9_WGS=128";; w192) E="SV_WGRAD9_WGS=192";; w256) E="SV_WGRAD9_WGS=256";; long300) E="SV_WGRAD9_LONG_GFLOP=300";; esac
    env $E timeout -k 10 300 python bench.py --backbone convnext_large --batch 64 --steps 5 --warmup 2 --no-cpu-baseline > $O/l_${v}_$i.json 2>>$O/bench.err || exit $?
    python -c "import json; d=json.loads(open('$O/l_${v}_$i.json').read().strip().splitlines()[-1]); print('$v $E', d['value'], d['ms_per_step'])"
  done
done
