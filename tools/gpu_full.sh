#!/bin/bash
# Round-end style GPU session: parity tests + smoke + default bench (PMC passes inside) + kernel trace, then the
# SQ counter passes.  Usage: tools/gpu_full.sh TAG
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
TAG=$1
bash tools/gpu_session.sh "$TAG" || exit $?
bash tools/gpu_pmc.sh "$TAG" \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU" \
  "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
  > "gpurun_out/$TAG/pmc_sq.txt" 2>&1
rc=$?
tail -80 "gpurun_out/$TAG/pmc_sq.txt"
exit $rc
