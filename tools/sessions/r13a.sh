#!/bin/bash
# round 6, first GPU call: the whole GPU suite on the round's correctness fixes (mlp_fwd unconditional weight DMA, dw+LN
# statistics barrier, head-loss poison, BN fold acq_rel, stream-exact bucket readiness, the ISA markers), then the
# cross-lane mlpb128 build's run-to-run test (libsv_kernels_xl.so, -DSV_MLPB_XLANE=1: the test names what differs),
# then the default training line and the classification line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOTDIR=$(pwd)
N=${1:-r13a}
O=$ROOTDIR/gpurun_out/$N
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
SV_LIB_PATH=$ROOTDIR/spine-vision_amd/libsv_kernels_xl.so timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_mlp_fused_gpu.py -k "bwd_fused_matches" > $O/xl_tests.log 2>&1
echo "xlane build: exit $?"; grep -E "passed|failed|differs" $O/xl_tests.log | head -10
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('train', d['value'], d['ms_per_step'])"
timeout -k 10 300 python bench.py --workload classification --steps 30 --warmup 5 --no-cpu-baseline > $O/bench_cls.json 2>/dev/null || exit 1
python -c "import json; d=json.loads(open('$O/bench_cls.json').read().strip().splitlines()[-1]); print('cls', d['value'], d['ms_per_step'])"
