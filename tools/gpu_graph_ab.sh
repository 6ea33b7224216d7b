#!/bin/bash
# classification step: graph-replay parity tests, then bench A/B of --graph on/off (interleaved, 2 rounds)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-graphab}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_trainer_gpu.py tests/test_abi.py -q -x --timeout 120 --timeout-method thread -k "${TK:-graphed or abi}" > "$OUT/tests.log" 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $OUT/tests.log)"
[ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" "$OUT/tests.log" | head -20; exit $rc; }
for r in 1 2; do
  for gr in on off; do
    timeout -k 10 300 python bench.py --workload classification --steps 30 --warmup 5 --no-cpu-baseline --graph $gr > "$OUT/bench_${gr}_$r.json" 2> "$OUT/bench_${gr}_$r.err"
    rc=$?; echo "graph=$gr r=$r rc=$rc $(python -c "import json; d=json.load(open('$OUT/bench_${gr}_$r.json')); print(d['value'], d['ms_per_step'], d['config']['hip_graph'])" 2>&1)"
    [ $rc -ne 0 ] && { tail -5 "$OUT/bench_${gr}_$r.err"; exit $rc; }
  done
done
exit 0
