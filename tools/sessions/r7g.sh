#!/bin/bash
# round 4: full GPU suite on the current tree, then the localization and classification lines
set -u
O=gpurun_out/r7g
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -q -rf --timeout 600 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 $O/tests.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench.json 2>$O/bench.err || exit $?
timeout -k 10 300 python bench.py --workload classification --steps 30 --warmup 5 --no-cpu-baseline > $O/cls.json 2>>$O/bench.err || exit $?
SV_WGRAD9_WGS=256 timeout -k 10 300 python bench.py --workload classification --steps 30 --warmup 5 --no-cpu-baseline > $O/cls_wgs256.json 2>>$O/bench.err || exit $?
for f in bench cls cls_wgs256; do python -c "import json; d=json.load(open('$O/$f.json')); print('$f', d['value'], d['ms_per_step'])"; done
