#!/bin/bash
# SQ counters of the chain's kernels for each library given (exp_ab/lib<name>.so swapped in, product restored)
set -o pipefail
cd "$(dirname "$0")/../../.."
cp gr-dvbt2ll_amd/dvbt2ll/libdvbt2ll_hip.so /tmp/prod.so
rc=0
for v in "$@"; do
  cp exp_ab/lib$v.so gr-dvbt2ll_amd/dvbt2ll/libdvbt2ll_hip.so
  bash tools/gpu_pmc.sh $v "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE" "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA" > gpurun_out/pmc_$v.txt 2>&1 || { rc=$?; break; }
done
cp /tmp/prod.so gr-dvbt2ll_amd/dvbt2ll/libdvbt2ll_hip.so
exit $rc
