#!/bin/bash
# round 4: comm start latency with the 128-workgroup weight gradients, and the step cost of the 32-CU cap reserve
set -u
O=gpurun_out/r7h
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q -s --timeout 200 --timeout-method thread tests/test_comm_reserve_gpu.py > $O/comm.log 2>&1
grep "\[comm\]" $O/comm.log
for i in 1 2; do
  for r in 0 32; do
    SV_BENCH_RESERVE=$r timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/res${r}_$i.json 2>>$O/bench.err || exit $?
    python -c "import json; d=json.load(open('$O/res${r}_$i.json')); print('reserve $r', d['value'], d['ms_per_step'])"
  done
done
