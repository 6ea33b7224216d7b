#!/bin/bash
# round 3, session 3 measurement set on the final tree: full -m gpu suite + smoke, the default bench line (with
# cpu_baseline), classification line, rocprof kernel stats of the default bench, PMC classes (traffic, MFMA busy)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r5z}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
TESTS=1 bash tools/gpu_measure.sh "$TAG" || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 $OUT/smoke.txt)"; [ $rc -ne 0 ] && exit $rc
CLOCK=0 bash tools/gpu_pmc.sh "$TAG/pmc"
