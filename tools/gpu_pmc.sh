#!/bin/bash
# PMC passes over a short default bench run (kernel-trace only, one counter group per pass, each its own
# run): FETCH_SIZE, WRITE_SIZE (traffic), MFMA busy + GRBM (utilisation, effective clock); then the
# per-class summary (tools/pmc_classes.py) and the in-kernel clock of the v9 GEMM (tools/clock_stamp.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-pmc}
BENCH_ARGS=${BENCH_ARGS:-}
CFG=${CFG:-convnext_base/512/bs32/bf16}
mkdir -p "$OUT"
ROOTDIR=$(pwd)
cd /tmp && export TMPDIR=/tmp
i=0
while read -r name ctrs; do
  [ -z "$name" ] && continue
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctrs --output-format csv -d "$ROOTDIR/$OUT/pmc_$name" -o run -- python3 "$ROOTDIR/bench.py" --steps 2 --warmup 1 --no-cpu-baseline $BENCH_ARGS > "$ROOTDIR/$OUT/pmc_$name.log" 2>&1
  rc=$?; echo "pmc $name rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done <<< "FETCH_SIZE FETCH_SIZE
WRITE_SIZE WRITE_SIZE
MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
cd "$ROOTDIR"
python3 tools/pmc_classes.py "$OUT" "$CFG" --json "$OUT/pmc_classes.json" > "$OUT/pmc_classes.txt" 2>&1
rc=$?; echo "classes rc=$rc"
[ $rc -ne 0 ] && exit $rc
if [ "${CLOCK:-1}" = "1" ]; then
  timeout -k 10 120 python3 tools/clock_stamp.py > "$OUT/clock_stamp.txt" 2>&1
  rc=$?; echo "clock rc=$rc"; tail -3 "$OUT/clock_stamp.txt"
fi
exit 0
