#!/bin/bash
# PMC counter passes (kernel-trace only, one group per pass) over a filtered gemm_bench run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-pmc}
mkdir -p "$OUT"
ROOTDIR=$(pwd)
ARGS=${GB_ARGS:---stages S1 --cases fc1_fwd(dual) --iters 5}
cd /tmp && export TMPDIR=/tmp
i=0
while read -r ctrs; do
  [ -z "$ctrs" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctrs --output-format csv -d "$ROOTDIR/$OUT/p$i" -o run -- python3 "$ROOTDIR/tools/gemm_bench.py" $ARGS > "$ROOTDIR/$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i ($ctrs) rc=$rc" | tee -a "$ROOTDIR/$OUT/status"
  [ $rc -ne 0 ] && exit $rc
done <<< "${PMC_SETS:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES
SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU
TCC_EA0_WRREQ TCC_EA0_WRREQ_64B TCC_EA0_WRREQ_STALL TCC_TOO_MANY_EA_WRREQS_STALL
TCC_EA0_RDREQ TCC_EA0_RDREQ_DRAM TCC_HIT TCC_MISS
TA_BUSY_avr TCP_TCP_TA_DATA_STALL_CYCLES TCP_PENDING_STALL_CYCLES TA_TOTAL_WAVEFRONTS}"
exit 0
