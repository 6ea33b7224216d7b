#!/bin/bash
# round 5, first GPU call: the advisor fixes (split-7 spread fold, ResNet bf16 absolute bounds), the renamed comm
# latency test (dumps gpurun_out/comm_latency.json), then the default bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r10a}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_gemm_family_gpu.py::test_wgrad_inkernel_fold_bitwise" \
  tests/test_resnet_parity_256_gpu.py tests/test_comm_reserve_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "PASS|FAIL|\[parity\]|\[comm\]" $O/tests.log | tail -40
cp gpurun_out/comm_latency.json $O/ 2>/dev/null
timeout -k 10 600 python bench.py > $O/bench.json 2>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline'])"
