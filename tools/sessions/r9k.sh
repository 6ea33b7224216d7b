#!/bin/bash
# round 4: per-stage GEMM family sweep (auto vs v2 / v3 / v8 / v9) on the ConvNeXt-base bs32 shapes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r9k}
mkdir -p $O
timeout -k 10 500 python tools/gemm_bench.py --stages S1,S2,S3,S4 --iters 10 --impls 0,2,3,8,9 \
  --cases "fc1_fwd(dual),fc2_fwd,fc2_dgrad(mul),fc1_dgrad,fc1_wgrad,fc2_wgrad+bias" > $O/sweep.txt 2>&1
rc=$?; cat $O/sweep.txt | tail -40; exit $rc
