#!/bin/bash
# round 5 final lines: BatchNorm / ResNet tests after the hoisted-parameter kernels, the default bench (CPU baseline in
# the run), the classification line (30 steps) with its kernel trace / queue breakdown, the eval line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOTDIR=$(pwd)
N=${1:-r11u}
O=$ROOTDIR/gpurun_out/$N
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_resnet_gpu.py tests/test_bn_small_gpu.py tests/test_bn_fold_gpu.py tests/test_head_loss_gpu.py tests/test_bs32_parity_gpu.py::test_resnet50_256_bs32_bf16_step > $O/t.log 2>&1 || { grep -E "FAIL|Error|assert" $O/t.log | head -20; tail -20 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
head -c 300 $O/bench.json; echo
timeout -k 10 300 python bench.py --workload classification --steps 30 --warmup 5 --no-cpu-baseline > $O/bench_cls.json 2>/dev/null || exit 1
head -c 200 $O/bench_cls.json; echo
timeout -k 10 300 python bench.py --inference --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_inf.json 2>/dev/null || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/cls_trace" -o run -- python3 "$ROOTDIR/bench.py" --workload classification --steps 3 --warmup 2 --no-cpu-baseline > "$O/cls_trace_bench.json" 2> "$O/cls_trace.err" || exit 1
cd "$ROOTDIR"
KT=$(find $O/cls_trace -name "*kernel_trace.csv" | head -1)
python tools/queue_breakdown.py $KT 25 > $O/cls_queues.txt && head -3 $O/cls_queues.txt
gzip -f $KT
