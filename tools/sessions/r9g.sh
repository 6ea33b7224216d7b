#!/bin/bash
# round 4: sv_ctx (ABI v4) on the GPU, kernel + engine tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r9g}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_trainer_gpu.py tests/test_ddp_gpu.py tests/test_resnet_parity_256_gpu.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; exit $rc
