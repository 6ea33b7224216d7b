#!/bin/bash
# PMC counter passes (kernel-trace only, one counter group per pass, each pass its own run) over an
# arbitrary python command:  CMD="tools/dw_bench.py --stages S3 --iters 3" bash tools/pmc_run.sh OUT
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-pmc}
mkdir -p "$OUT"
ROOTDIR=$(pwd)
cd /tmp && export TMPDIR=/tmp
i=0
while read -r ctrs; do
  [ -z "$ctrs" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctrs --output-format csv -d "$ROOTDIR/$OUT/p$i" -o run -- python3 $ROOTDIR/$CMD > "$ROOTDIR/$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i ($ctrs) rc=$rc" | tee -a "$ROOTDIR/$OUT/status"
  [ $rc -ne 0 ] && exit $rc
done <<< "${PMC_SETS:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES
SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES
FETCH_SIZE
WRITE_SIZE
TCC_HIT TCC_MISS GRBM_GUI_ACTIVE GRBM_COUNT}"
exit 0
