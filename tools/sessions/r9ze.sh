#!/bin/bash
# round 4: per-class upper bounds in the ConvNeXt-base step: each class's launches skipped (SV_DIAG_SKIP, timing only)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r9ze}
mkdir -p $O
for i in 1 2; do
  for v in none dw_fwd dw_bwd_data dw_wgrad ln_bwd adamw; do
    if [ $v = none ]; then E=""; else E=$v; fi
    SV_DIAG_SKIP=$E timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_${v}_$i.json 2>>$O/bench.err || exit $?
    python -c "import json; d=json.loads(open('$O/b_${v}_$i.json').read().strip().splitlines()[-1]); print('skip=$v', d['value'], d['ms_per_step'])"
  done
done
