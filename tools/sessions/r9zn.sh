#!/bin/bash
# round 4: wgrad workgroup target 128 vs 256 with bf16 slabs: ConvNeXt-base, classification, ConvNeXt-large
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r9zn}
mkdir -p $O
for i in 1 2 3; do
  for v in 128 256; do
    SV_WGRAD9_WGS=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_${v}_$i.json 2>>$O/bench.err || exit $?
    SV_WGRAD9_WGS=$v timeout -k 10 300 python bench.py --workload classification --steps 30 --warmup 5 --no-cpu-baseline > $O/c_${v}_$i.json 2>>$O/bench.err || exit $?
    python -c "import json; d=json.loads(open('$O/b_${v}_$i.json').read().strip().splitlines()[-1]); c=json.loads(open('$O/c_${v}_$i.json').read().strip().splitlines()[-1]); print('wgs=$v base', d['value'], 'cls', c['value'])"
  done
done
for v in 128 256; do
  SV_WGRAD9_WGS=$v timeout -k 10 300 python bench.py --backbone convnext_large --batch 64 --steps 5 --warmup 2 --no-cpu-baseline > $O/l_${v}.json 2>>$O/bench.err || exit $?
  python -c "import json; d=json.loads(open('$O/l_${v}.json').read().strip().splitlines()[-1]); print('wgs=$v large', d['value'])"
done
