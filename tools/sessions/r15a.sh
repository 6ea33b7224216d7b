#!/bin/bash
# round 6 (final session): cross-lane fused-MLP-backward bisection (which butterfly makes dz differ run to run), the
# whole GPU suite, smoke, the default bench (now with the configs[3] classification line)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r15a}
mkdir -p $O
for v in "" _xl1 _xl2 _xl3; do
  SV_LIB_PATH=$PWD/spine-vision_amd/libsv_kernels$v.so timeout -k 10 180 python -u tools/mlp_bwd_diag.py 524288 524288 > $O/diag$v.txt 2>&1 || { tail -20 $O/diag$v.txt; exit 1; }
  echo "== lib$v"; grep "deterministic\|differing" $O/diag$v.txt
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.txt 2>&1 || { tail -30 $O/suite.txt; exit 1; }
tail -2 $O/suite.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -3 $O/smoke.txt
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); c=d.get('configs3_classification',{}); print('train', d['value'], d['ms_per_step'], d['roofline']['frac'], 'mainq', (d.get('main_queue') or {}).get('busy_ms_per_step'), 'cls', c.get('value'), c.get('error'))"
