#!/bin/bash
# round 6 (re-entry): SV_DEFER_WGRAD_FLUSH (a ResNet block's side-stream weight gradients enqueued after the next
# block's first BatchNorm backward pass) -- bitwise test, then the classification line A/B interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r16c}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_trainer_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "deferred_wgrad_flush or graph_forward_matches" > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -2 $O/t.txt
for v in 0 1 0 1; do
  SV_DEFER_WGRAD_FLUSH=$v timeout -k 10 300 python -u bench.py --workload classification --steps 30 --warmup 5 --no-cpu-baseline > $O/cls_$v.json 2> $O/cls.err || { tail -20 $O/cls.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/cls_$v.json').read().strip().splitlines()[-1]); print('defer $v', d['value'], d['ms_per_step'], (d.get('main_queue') or {}).get('busy_ms_per_step'))"
done
for v in 0 1; do
  SV_DEFER_WGRAD_FLUSH=$v timeout -k 10 300 python -u bench.py --workload classification --backbone resnet18 --steps 30 --warmup 5 --no-cpu-baseline > $O/r18_$v.json 2> $O/cls.err || { tail -20 $O/cls.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/r18_$v.json').read().strip().splitlines()[-1]); print('r18 defer $v', d['value'], d['ms_per_step'])"
done
