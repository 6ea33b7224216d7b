#!/bin/bash
# round 4: transposed gather wgrad (stem, layer1 3x3) at 3 ring stages / 512 workgroups (w4s3) vs 4 / 256 (base)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r8k}
mkdir -p $O
for v in base w4s3 base w4s3; do
  if [ $v = base ]; then L=""; else L=$(pwd)/spine-vision_amd/libsv_kernels_$v.so; fi
  SV_LIB_PATH=$L timeout -k 10 120 python tools/conv_bench.py --iters 20 --only l1_3x3 >> $O/conv_$v.txt 2>&1 || exit $?
  SV_LIB_PATH=$L timeout -k 10 120 python tools/conv_bench.py --iters 20 --only stem >> $O/conv_$v.txt 2>&1 || exit $?
done
grep -h "wgrad" $O/conv_base.txt $O/conv_w4s3.txt
for i in 1 2 3; do
  for v in base w4s3; do
    if [ $v = base ]; then L=""; else L=$(pwd)/spine-vision_amd/libsv_kernels_$v.so; fi
    SV_LIB_PATH=$L timeout -k 10 300 python bench.py --workload classification --steps 50 --warmup 10 --no-cpu-baseline > $O/cls_${v}_$i.json 2>>$O/bench.err || exit $?
    python -c "import json; d=json.loads(open('$O/cls_${v}_$i.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
  done
done
