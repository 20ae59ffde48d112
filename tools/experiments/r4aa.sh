set -o pipefail
mkdir -p gpurun_out/r4aa
start=$(date +%s)
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4aa/bench.json 2> gpurun_out/r4aa/bench.err; rc=$?
echo "bench rc=$rc seconds=$(( $(date +%s) - start ))"
exit $rc
