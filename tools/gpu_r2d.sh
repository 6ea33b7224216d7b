#!/bin/bash
# round-2: golden-trainer tests + the tests changed since r2c, then the suite and the bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r2d}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_golden_r2_gpu.py "tests/test_resnet_gpu.py::test_resnet_block_backward_teacher_forced" tests/test_parity_geometry_gpu.py tests/test_ddp_gpu.py > "$OUT/new.log" 2>&1
rc=$?; echo "new rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > "$OUT/gpu_suite.log" 2>&1
rc=$?; echo "suite rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; exit $rc
