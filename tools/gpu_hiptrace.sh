#!/bin/bash
# HIP API trace of a short bench run (host-side stalls: synchronising calls, allocations per step)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-ht}
mkdir -p "$OUT"
ROOTDIR=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d "$ROOTDIR/$OUT/prof" -o run -- python3 "$ROOTDIR/bench.py" --steps 5 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > "$ROOTDIR/$OUT/bench.json" 2> "$ROOTDIR/$OUT/prof.err"
rc=$?; echo "rocprof rc=$rc"
exit $rc
