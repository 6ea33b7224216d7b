#!/bin/bash
# round-2 check: new parity / RCCL tests, then the whole GPU suite, then the bench (default and --gpus 1)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r2b}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_parity_geometry_gpu.py tests/test_ddp_gpu.py > "$OUT/parity.log" 2>&1
rc=$?; echo "parity rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > "$OUT/gpu_suite.log" 2>&1
rc=$?; echo "suite rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; exit $rc
