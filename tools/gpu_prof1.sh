set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/prof/trace -o bench -- python3 bench.py --steps 10 --warmup 2 --no-pmc --no-cpu-baseline > gpurun_out/prof/trace_bench.json 2> gpurun_out/prof/trace.err
echo "TRACE EXIT $?"
for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE"; do
  tag=$(echo $set | tr ' ' '_' | cut -c1-40)
  timeout -k 10 240 rocprofv3 --pmc $set -T -f csv -d gpurun_out/prof/pmc_$tag -o pmc -- python3 bench.py --pmc-child --steps 2 --warmup 1 > /dev/null 2> gpurun_out/prof/pmc_$tag.err
  echo "PMC $tag EXIT $?"
done
find gpurun_out/prof -name "*.csv" | head -30
