#!/bin/bash
# ResNet iteration: conv/BN/trainer parity tests, conv pass timings, classification bench A/B of the
# side-stream weight gradients (interleaved, two rounds), one rocprof kernel-stats pass
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-clsab}
mkdir -p "$OUT"
ROOTDIR=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_resnet_gpu.py tests/test_trainer_gpu.py "tests/test_parity_geometry_gpu.py" -q -x --timeout 120 --timeout-method thread -k "${TK:-not convnext}" > "$OUT/tests.log" 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $OUT/tests.log)"
[ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" "$OUT/tests.log" | head -20; exit $rc; }
timeout -k 10 120 python tools/conv_bench.py > "$OUT/conv.txt" 2>&1 || exit $?
for r in 1 2; do
  for ss in 1 0; do
    SV_SIDE_STREAM=$ss timeout -k 10 300 python bench.py --workload classification --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_ss${ss}_$r.json" 2> "$OUT/bench_ss${ss}_$r.err"
    rc=$?; echo "side=$ss r=$r rc=$rc $(head -c 150 $OUT/bench_ss${ss}_$r.json | cut -c100-150)"
    [ $rc -ne 0 ] && exit $rc
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOTDIR/$OUT/prof" -o run -- python3 "$ROOTDIR/bench.py" --workload classification --steps 3 --warmup 2 --no-cpu-baseline > "$ROOTDIR/$OUT/prof_bench.json" 2> "$ROOTDIR/$OUT/prof.err"
rc=$?; echo "rocprof rc=$rc"
exit $rc
