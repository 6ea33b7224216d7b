#!/bin/bash
# round 6: the per-block main -> side hand-off through events without the system-scope fence (native.handoff):
# the bitwise schedule / parity tests and the DDP tests, the training line A/B (SV_FENCELESS_EVENTS 1 / 0,
# interleaved), the trace's main-queue gaps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOTDIR=$(pwd)
N=${1:-r13p}
O=$ROOTDIR/gpurun_out/$N
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_parity_geometry_gpu.py tests/test_ddp_gpu.py tests/test_bs32_parity_gpu.py > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | head -20; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for f in 1 0 1 0; do
  SV_FENCELESS_EVENTS=$f timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$f.json 2> $O/bench_$f.err || { tail -5 $O/bench_$f.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_$f.json').read().strip().splitlines()[-1]); print('fenceless=$f train', d['value'], d['ms_per_step'], d['main_queue']['busy_ms_per_step'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/prof" -o run -- python3 "$ROOTDIR/bench.py" --steps 3 --warmup 2 --no-cpu-baseline > "$O/prof_bench.json" 2> "$O/prof.err" || { tail -20 "$O/prof.err"; exit 1; }
cd "$ROOTDIR"
KT=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python tools/queue_gaps.py $KT 15 > $O/gaps.txt; tail -14 $O/gaps.txt
gzip -f $KT
