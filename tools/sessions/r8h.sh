#!/bin/bash
# round 4: ConvNeXt-base bs32 step A/B: nt loads of the GELU-grad epilogue operand (auxnt) and of the wgrad B operand (slabbnt)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r8g}
mkdir -p $O
for i in 1 2 3; do
  for v in base auxnt slabbnt; do
    if [ $v = base ]; then L=""; else L=$(pwd)/spine-vision_amd/libsv_kernels_$v.so; fi
    SV_LIB_PATH=$L timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/${v}_$i.json 2>>$O/bench.err || exit $?
    python -c "import json; d=json.loads(open('$O/${v}_$i.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
  done
done
