#!/bin/bash
# round 6: AdamW overlapped with the next forward (SV_OPT_OVERLAP=1, StepEngine(overlap_optimizer)): bitwise tests, step
# digests of both engines, then the default bench line interleaved against it
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOTDIR=$(pwd)
N=${1:-r14b}
O=$ROOTDIR/gpurun_out/$N
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_opt_overlap_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
for f in 0 1; do
  SV_OPT_OVERLAP=$f timeout -k 10 300 python tools/step_digest.py --workload localization --steps 3 > $O/digest_$f.json 2> $O/digest_$f.err || { tail -5 $O/digest_$f.err; exit 1; }
  cat $O/digest_$f.json
done
for f in 1 0 1 0; do
  SV_OPT_OVERLAP=$f timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$f.json 2> $O/bench_$f.err || { tail -5 $O/bench_$f.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_$f.json').read().strip().splitlines()[-1]); print('overlap=$f train', d['value'], d['ms_per_step'], d['main_queue']['busy_ms_per_step'])"
done
