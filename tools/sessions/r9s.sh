#!/bin/bash
# round 4: nt cache policy on the fc1 GELU-dual epilogue's GELU(h) store (SV_G9_C2_CPOL=2 build) vs the default
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r9s}
mkdir -p $O
for i in 1 2 3; do
  for v in def c2nt; do
    if [ $v = def ]; then L=""; else L=$(pwd)/spine-vision_amd/libsv_kernels_c2nt.so; fi
    SV_LIB_PATH=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_${v}_$i.json 2>>$O/bench.err || exit $?
    python -c "import json; d=json.loads(open('$O/b_${v}_$i.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
  done
done
