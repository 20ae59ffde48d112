set -o pipefail
cp gr-dvbt2ll_amd/dvbt2ll/libdvbt2ll_hip.so /tmp/prod.so
cp exp_ab/libr6fused.so gr-dvbt2ll_amd/dvbt2ll/libdvbt2ll_hip.so
bash tools/gpu_pmc.sh r6f "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE" "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" "SQ_VALU_MFMA_BUSY_CYCLES" > gpurun_out/pmc_r6f.txt 2>&1
rc=$?
cp /tmp/prod.so gr-dvbt2ll_amd/dvbt2ll/libdvbt2ll_hip.so
exit $rc
