#!/bin/bash
# SQ counters of every other config's kernels (tools/gpu_pmc.sh over bench.py --pmc-child --config c)
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
for c in cfg1 cfg2 cfg4 cfg5; do
  PMC_ARGS="--config $c" bash tools/gpu_pmc.sh sq_$c "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE" "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" > gpurun_out/sq_$c.txt 2>&1 || { tail -5 gpurun_out/sq_$c.txt; exit 1; }
  echo "config $c done"
done
