#!/bin/bash
# round 4: persistent wgrad workgroup target with bf16 slabs (SV_WGRAD9_WGS), ConvNeXt-base bs32
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r9zm}
mkdir -p $O
for i in 1 2; do
  for v in 128 160 192 256; do
    SV_WGRAD9_WGS=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_${v}_$i.json 2>>$O/bench.err || exit $?
    python -c "import json; d=json.loads(open('$O/b_${v}_$i.json').read().strip().splitlines()[-1]); print('wgs=$v', d['value'], d['ms_per_step'])"
  done
done
