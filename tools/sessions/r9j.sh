#!/bin/bash
# round 4: no split-K for the strided dgrads (SV_S2_NOSPLIT) with the BatchNorm statistics from their own pass
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r9j}
mkdir -p $O
for i in 1 2 3 4; do
  for v in b d; do
    case $v in a) E="SV_S2_BN=1 SV_S2_NOSPLIT=0";; b) E="SV_S2_BN=0 SV_S2_NOSPLIT=0";; d) E="SV_S2_BN=0 SV_S2_NOSPLIT=1";; esac
    env $E timeout -k 10 300 python bench.py --workload classification --steps 50 --warmup 10 --no-cpu-baseline > $O/cls_${v}_$i.json 2>>$O/bench.err || exit $?
    python -c "import json; d=json.loads(open('$O/cls_${v}_$i.json').read().strip().splitlines()[-1]); print('$v $E', d['value'], d['ms_per_step'])"
  done
done
