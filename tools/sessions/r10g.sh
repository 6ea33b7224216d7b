#!/bin/bash
# round 5: fused MLP with two 4-wave workgroups per CU at C = 128 -- bitwise tests + standalone timing
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r10g}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_mlp_fused_gpu.py > $O/t_mlp.log 2>&1 || { tail -40 $O/t_mlp.log; exit 1; }
grep -cE "PASSED" $O/t_mlp.log
timeout -k 10 300 python tools/mlp_bench.py --shapes base-S1,base-S2,large-S1 > $O/mlp_bench.txt 2>&1 || { tail -20 $O/mlp_bench.txt; exit 1; }
cat $O/mlp_bench.txt
