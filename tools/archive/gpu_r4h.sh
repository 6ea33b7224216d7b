#!/bin/bash
# round 3 measurement set: default bench line (+ cpu_baseline), classification line, DataLoader-fed trainer
# lines (device / host transform), rocprof kernel stats of the default line, PMC passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r4h}
mkdir -p "$OUT"
ROOTDIR=$(pwd)
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc $(head -c 200 $OUT/bench.json)"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --workload classification --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_cls.json" 2> "$OUT/bench_cls.err"
rc=$?; echo "cls rc=$rc $(head -c 200 $OUT/bench_cls.json)"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --trainer --steps 60 > "$OUT/trainer_device.json" 2> "$OUT/trainer_device.err"
rc=$?; echo "trainer device rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/trainer_device.err"; exit $rc; }
timeout -k 10 400 python bench.py --trainer --steps 30 --transform host > "$OUT/trainer_host.json" 2> "$OUT/trainer_host.err"
rc=$?; echo "trainer host rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/trainer_host.err"; exit $rc; }
timeout -k 10 300 python tools/host_time.py > "$OUT/host_time.txt" 2>&1
echo "host_time rc=$? $(tail -2 $OUT/host_time.txt)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOTDIR/$OUT/prof" -o run -- python3 "$ROOTDIR/bench.py" --steps 3 --warmup 2 --no-cpu-baseline > "$ROOTDIR/$OUT/prof_bench.json" 2> "$ROOTDIR/$OUT/prof.err"
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && exit $rc
cd "$ROOTDIR"
CLOCK=0 bash tools/gpu_pmc.sh "$(basename $OUT)/pmc"
