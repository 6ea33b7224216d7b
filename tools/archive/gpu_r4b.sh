#!/bin/bash
# round 3, session 1: new parity / ADVICE / comm-reserve tests, the default bench line, PMC classes + clock
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r4b}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_resize_gpu.py tests/test_resnet_parity_256_gpu.py tests/test_comm_reserve_gpu.py tests/test_trainer_gpu.py -k "resize or resnet50_256 or comm or rebound or two_forwards or graph" > "$OUT/tests.log" 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $OUT/tests.log)"
[ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" "$OUT/tests.log" | head -20; exit $rc; }
timeout -k 10 400 python bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc $(head -c 300 $OUT/bench.json)"
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_pmc.sh "$(basename $OUT)/pmc"
