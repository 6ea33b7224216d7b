#!/bin/bash
# round 4: with the whole-chip wgrads -- side-stream wave priority (SV_SIDE_PRIO) and the side stream itself
# (SV_SIDE_STREAM=0), ConvNeXt-base bs32 interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r9zs}
mkdir -p $O
for i in 1 2; do
  for v in def prio0 noside; do
    case $v in def) E="SV_SIDE_PRIO=1";; prio0) E="SV_SIDE_PRIO=0";; noside) E="SV_SIDE_STREAM=0";; esac
    env $E timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_${v}_$i.json 2>>$O/bench.err || exit $?
    python -c "import json; d=json.loads(open('$O/b_${v}_$i.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
  done
done
