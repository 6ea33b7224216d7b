#!/bin/bash
# round 4: ConvNeXt block wgrads at the whole-chip target (SV_CNX_WGRAD_WGS, default 256) -- parity and step A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r9zo}
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q -s --timeout 400 --timeout-method thread tests/test_bs32_parity_gpu.py tests/test_backbone_gpu.py tests/test_parity_geometry_gpu.py tests/test_golden_gpu.py tests/test_ddp_gpu.py > $O/tests.log 2>&1
rc=$?; grep "\[parity\] convnext" $O/tests.log; tail -1 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for v in 256 128; do
    SV_CNX_WGRAD_WGS=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_${v}_$i.json 2>>$O/bench.err || exit $?
    python -c "import json; d=json.loads(open('$O/b_${v}_$i.json').read().strip().splitlines()[-1]); print('cnx_wgs=$v', d['value'], d['ms_per_step'])"
  done
done
