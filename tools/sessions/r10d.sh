#!/bin/bash
# round 5: PMC passes over the fused MLP standalone bench (S1): issue / wait split, VALU and MFMA busy, LDS conflicts
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=r10d
PMC_SETS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_WR
GRBM_GUI_ACTIVE GRBM_COUNT" CMD="tools/mlp_bench.py --shapes base-S1 --iters 3" bash tools/pmc_run.sh $O || exit 1
python tools/pmc_dump.py gpurun_out/$O mlp_fwd gemm9
