#!/bin/bash
# round 3, session 3: split-K depth of the side-stream wgrads (SV_WGRAD9_WGS = workgroups per wgrad launch:
# 256 default, 128, 64 -> fewer f32 slabs to fold) interleaved, and a kernel + memory-copy trace of two steps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r5f}
mkdir -p "$OUT"
ROOTDIR=$(pwd)
for r in 1 2; do
  for v in 256 128 64; do
    SV_WGRAD9_WGS=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_${v}_$r.json" 2> "$OUT/bench_${v}_$r.err"
    rc=$?; echo "bench wgs=$v $r rc=$rc $(python3 -c "import json; d=json.load(open('$OUT/bench_${v}_$r.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], 'wgrad', r['kernels']['wgrad']['avg_launch_us'], 'fold', r['kernels']['fold']['ms_per_step'])" 2>/dev/null)"
    [ $rc -ne 0 ] && exit $rc
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$ROOTDIR/$OUT/trace" -o run -- python3 "$ROOTDIR/bench.py" --steps 2 --warmup 2 --no-cpu-baseline > "$ROOTDIR/$OUT/trace.json" 2> "$ROOTDIR/$OUT/trace.err"
rc=$?; echo "trace rc=$rc"
exit $rc
