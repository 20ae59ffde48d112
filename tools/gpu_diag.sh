set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/diag
bash tools/gpu_o32_phases.sh cfg3 > gpurun_out/diag/phases.txt 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES -T -f csv -d gpurun_out/diag/pmc_waves -o pmc -- python bench.py --pmc-child --steps 1 --warmup 1 > gpurun_out/diag/pmc_waves.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d gpurun_out/diag/pmc_wr -o pmc -- python bench.py --pmc-child --steps 1 --warmup 1 > gpurun_out/diag/pmc_wr.log 2>&1
echo done
