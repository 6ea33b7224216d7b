#!/bin/bash
# round 6: the K = 512 epilogue-heavy GEMMs of S3 / S2 standalone on each kernel family (impl 9 / 3 / 8 / 2), hipBLASLt
# beside them (plain store) -- is a two-workgroup-per-CU family better where the epilogue dominates?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOTDIR=$(pwd)
N=${1:-r13v}
O=$ROOTDIR/gpurun_out/$N
mkdir -p $O
timeout -k 10 500 python -u tools/gemm_bench.py --stages S3,S2 --impls 9,3,8,2 --cases "fc1_fwd(dual),fc2_fwd,fc2_dgrad(mul),fc1_dgrad,torch_fc1_fwd,torch_fc2_fwd" > $O/gemm.txt 2>&1 || { tail -20 $O/gemm.txt; exit 1; }
cat $O/gemm.txt
