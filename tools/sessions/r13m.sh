#!/bin/bash
# round 6: matrix-core depthwise with the per-pass channel-group choice (fwd 16, bwd-data 32 at C <= 256 else 16), the
# eval forward on it, the weight gradient back on the VALU kernel (MFMA wgrad opt-in): dw tests, the whole GPU suite,
# the training line twice, the eval line, the classification line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOTDIR=$(pwd)
N=${1:-r13m}
O=$ROOTDIR/gpurun_out/$N
mkdir -p $O
timeout -k 10 900 python -u -m pytest --maxfail=8 -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1
echo "suite exit $?"; grep -E "^FAILED|[0-9]+ passed|failed" $O/tests.log | tail -10
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$i.json 2> $O/bench_$i.err || { tail -5 $O/bench_$i.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_$i.json').read().strip().splitlines()[-1]); k=d['roofline']['kernels']; print('train', d['value'], d['ms_per_step'], d['main_queue']['busy_ms_per_step'], {n: k[n]['ms_per_step'] for n in ('dw_fwd', 'dw_bwd_data', 'dw_wgrad')})"
done
timeout -k 10 300 python bench.py --inference --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_inf.json 2> $O/bench_inf.err || { tail -5 $O/bench_inf.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_inf.json').read().strip().splitlines()[-1]); print('eval', d['value'], d['ms_per_step'])"
SV_DW_MFMA=0 timeout -k 10 300 python bench.py --inference --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_inf_valu.json 2> $O/bench_inf_valu.err || { tail -5 $O/bench_inf_valu.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_inf_valu.json').read().strip().splitlines()[-1]); print('eval valu', d['value'], d['ms_per_step'])"
timeout -k 10 300 python bench.py --workload classification --steps 30 --warmup 5 --no-cpu-baseline > $O/bench_cls.json 2> $O/bench_cls.err || exit 1
python -c "import json; d=json.loads(open('$O/bench_cls.json').read().strip().splitlines()[-1]); print('cls', d['value'], d['ms_per_step'])"
