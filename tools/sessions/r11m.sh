#!/bin/bash
# round 5: ConvNeXt end-of-backward -- the last block's wgrads on the main stream (SV_TAIL_MAIN) and the lean
# release batch (SV_RELEASE_BATCH) A/B, after the schedule-knob bitwise test
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r11m}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread "tests/test_parity_geometry_gpu.py::test_convnext_bf16_schedule_knobs_match_default" > $O/t.log 2>&1 || { grep -E "FAIL|Error|assert" $O/t.log | head -20; tail -20 $O/t.log; exit 1; }
grep -c PASSED $O/t.log
for r in 1 2; do
for v in "0 4" "1 4" "1 64" "0 64"; do
  set -- $v
  SV_TAIL_MAIN=$1 SV_RELEASE_BATCH=$2 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_$1_$2_$r.json 2>>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_$1_$2_$r.json').read().strip().splitlines()[-1]); print('tail=$1 release=$2', d['value'], d['ms_per_step'], d.get('hbm_peak_allocated_gb'))"
done
done
