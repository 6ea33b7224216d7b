#!/bin/bash
# round 5: ResNet bf16 gradient stream -- kernel and block tests, ResNet floor / bs32 parity, classification bench
# with the stream on / off, rocprof kernel stats of the "on" line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOTDIR=$(pwd)
N=${1:-r11a}
O=gpurun_out/$N
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_resnet_gpu.py tests/test_bn_small_gpu.py ${RK:+-k "$RK"} > $O/t_resnet.log 2>&1 || { grep -E "FAIL|Error|assert" $O/t_resnet.log | head -30; tail -30 $O/t_resnet.log; exit 1; }
grep -c PASSED $O/t_resnet.log
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_resnet_parity_256_gpu.py tests/test_bs32_parity_gpu.py::test_resnet50_256_bs32_bf16_step tests/test_parity_geometry_gpu.py::test_resnet_bf16_side_stream_matches_single_stream > $O/t_parity.log 2>&1 || { grep -E "\[parity\]|FAIL|Error|assert" $O/t_parity.log | tail -30; exit 1; }
grep -E "\[parity\]|PASSED|rel" $O/t_parity.log | tail -30
for v in on off; do
  E=$([ $v = on ] && echo SV_RESNET_GRAD_BF16=1 || echo SV_RESNET_GRAD_BF16=0)
  env $E timeout -k 10 300 python bench.py --workload classification --steps 20 --warmup 5 --no-cpu-baseline > $O/b_$v.json 2>>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]); print('$v cls', d['value'], d['ms_per_step'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOTDIR/$O/prof" -o run -- python3 "$ROOTDIR/bench.py" --workload classification --steps 3 --warmup 2 --no-cpu-baseline > "$ROOTDIR/$O/prof_bench.json" 2> "$ROOTDIR/$O/prof.err" || { tail -20 "$ROOTDIR/$O/prof.err"; exit 1; }
find "$ROOTDIR/$O/prof" -name "*kernel_trace.csv" -delete
cd "$ROOTDIR"
python tools/stats_md.py $(find $O/prof -name "*kernel_stats.csv" | head -1) 3 "round 5 $N classification" "rocprofv3 --kernel-trace --stats -- python3 bench.py --workload classification --steps 3 --warmup 2 --no-cpu-baseline" 40 > $O/kernel_stats.md
head -30 $O/kernel_stats.md
