#!/bin/bash
# One bench line per BASELINE config shape on one GPU (final-tree record): ConvNeXt-base bs32 (the metric),
# ConvNeXt-large bs64, ResNet-50 3-head classification bs32, ConvNeXt-base eval forward, ResNet-18 bs32
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-cfg}
mkdir -p "$OUT"
run() {
  local name=$1; shift
  timeout -k 10 400 python bench.py "$@" --no-cpu-baseline > "$OUT/$name.json" 2> "$OUT/$name.err"
  local rc=$?
  echo "$name rc=$rc $(head -c 200 "$OUT/$name.json" | sed 's/.*"value": \([0-9.]*\).*/\1/')"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
run base --steps 10 --warmup 3
run large --backbone convnext_large --batch 64 --steps 5 --warmup 2
run cls --workload classification --steps 10 --warmup 3
run cls_r18 --workload classification --backbone resnet18 --steps 10 --warmup 3
run inf --inference --steps 10 --warmup 3
run inf_cls --workload classification --inference --steps 20 --warmup 5
run base2 --steps 10 --warmup 3
exit 0
