#!/bin/bash
# round 6 (re-entry): final-tree check of the pinned fused-MLP backward -- the whole GPU suite, smoke, the default
# bench (with the configs[3] line and the CPU baseline), a rocprofv3 kernel-trace summary of a short bench, and the
# pinned cross-lane build (SV_MLPB_XLANE=3) against the shipped shuffle form, interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r16a}
mkdir -p $O
SV_LIB_PATH=$PWD/spine-vision_amd/libsv_kernels_xl3.so timeout -k 10 240 python -u tools/mlp_bwd_diag.py 524288 524288 524288 > $O/diag_xl3p.txt 2>&1 || { tail -20 $O/diag_xl3p.txt; exit 1; }
grep "deterministic\|differing" $O/diag_xl3p.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.txt 2>&1 || { tail -30 $O/suite.txt; exit 1; }
tail -2 $O/suite.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -3 $O/smoke.txt
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); c=d.get('configs3_classification',{}); print('train', d['value'], d['ms_per_step'], d['roofline']['frac'], 'mainq', (d.get('main_queue') or {}).get('busy_ms_per_step'), 'cls', c.get('value'), c.get('error'))"
for v in "" _xl3 "" _xl3; do
  SV_BENCH_CLS=0 SV_LIB_PATH=$PWD/spine-vision_amd/libsv_kernels$v.so timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline > $O/ab$v.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/ab$v.json').read().strip().splitlines()[-1]); print('lib$v', d['value'], d['ms_per_step'])"
done
cd /tmp && SV_BENCH_CLS=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/prof_bench.json 2> $GRAFT_REPO_ROOT/$O/prof.err || { tail -20 $GRAFT_REPO_ROOT/$O/prof.err; exit 1; }
echo done
