#!/bin/bash
# round 6 (re-entry): config lines on the final tree, then the classification step's trace (queue breakdown, main-queue
# gaps: where the ResNet-50 step's idle main queue waits) and its host enqueue time
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_configs.sh r16b_configs || exit 1
bash tools/sessions/r13w.sh r16b_cls || exit 1
