#!/bin/bash
# round 6 (re-entry): final-tree GPU suite and smoke after the ResNet backward's opt-in enqueue knob
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r16d}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.txt 2>&1 || { tail -30 $O/suite.txt; exit 1; }
tail -2 $O/suite.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
