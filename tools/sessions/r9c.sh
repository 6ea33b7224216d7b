#!/bin/bash
# round 4: ConvNeXt-large bs64 with the nearest-to-target wgrad split (default, 128) vs a 256-workgroup target
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r9c}
mkdir -p $O
for i in 1 2; do
  for w in 128 256; do
    SV_WGRAD9_WGS=$w timeout -k 10 400 python bench.py --backbone convnext_large --batch 64 --steps 5 --warmup 2 --no-cpu-baseline > $O/large_w${w}_$i.json 2>>$O/bench.err || exit $?
    python -c "import json; d=json.loads(open('$O/large_w${w}_$i.json').read().strip().splitlines()[-1]); print('large wgs $w', d['value'], d['ms_per_step'], d['roofline']['kernels']['wgrad']['avg_launch_us'])"
  done
done
