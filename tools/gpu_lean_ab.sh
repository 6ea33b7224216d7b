#!/bin/bash
# ConvNeXt backward hand-off A/B: SV_LEAN_SYNC=1 (one main->side event per block, no record_stream) vs 0
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-lean}
mkdir -p "$OUT"
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q -rf --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
  rc=$?; echo "tests rc=$rc $(tail -1 $OUT/tests.log)"
  [ $rc -ne 0 ] && exit $rc
fi
for rep in 1 2; do
  for v in 1 0; do
    SV_LEAN_SYNC=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/l${v}_$rep.json" 2> "$OUT/l${v}_$rep.err"
    rc=$?; echo "lean=$v rep=$rep rc=$rc $(python -c "import json;b=json.load(open('$OUT/l${v}_$rep.json'));print(b['value'], b.get('hbm_reserved_gb'))")"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
