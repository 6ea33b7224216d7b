#!/bin/bash
# round 3: comm-reserve + trainer tests, the default bench line, the DataLoader-fed trainer lines, PMC classes + clock
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r4c}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_comm_reserve_gpu.py tests/test_trainer_gpu.py > "$OUT/tests.log" 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $OUT/tests.log)"
[ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" "$OUT/tests.log" | head -20; exit $rc; }
timeout -k 10 400 python bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc $(head -c 300 $OUT/bench.json)"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --trainer --steps 30 > "$OUT/trainer_device.json" 2> "$OUT/trainer_device.err"
rc=$?; echo "trainer device rc=$rc $(head -c 400 $OUT/trainer_device.json)"
[ $rc -ne 0 ] && { tail -20 "$OUT/trainer_device.err"; exit $rc; }
timeout -k 10 400 python bench.py --trainer --steps 20 --transform host > "$OUT/trainer_host.json" 2> "$OUT/trainer_host.err"
rc=$?; echo "trainer host rc=$rc $(head -c 400 $OUT/trainer_host.json)"
[ $rc -ne 0 ] && { tail -20 "$OUT/trainer_host.err"; exit $rc; }
bash tools/gpu_pmc.sh "$(basename $OUT)/pmc"
