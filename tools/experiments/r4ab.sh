set -o pipefail
BENCH_ARGS="--frames 192" NOPROBE=1 timeout -k 10 900 tools/experiments/gpu_ab.sh r4ab bbnocrc bbnopay bbnostore bbnostage
