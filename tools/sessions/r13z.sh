#!/bin/bash
# round 6: r13y (paired-column plane fill: parity, timing, ConvNeXt parity, training line) then r13x (the ResNet-50
# B=32 design check's printed distances)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/sessions/r13y.sh r13y || exit 1
bash tools/sessions/r13x.sh r13x
