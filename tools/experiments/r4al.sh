set -o pipefail
# data slots in bin order within each symbol half (no block-major runs, no bank_balance): the OFDM scatter's
# writes in bin order against the map's TI store losing its contiguous runs (planner-only variant); 192 frames
h=$(timeout -k 10 120 python tools/experiments/lib_iq_hash.py exp_build/libbinorder.so) && echo "binorder $h" &&
BENCH_ARGS="--frames 192" NOPROBE=1 timeout -k 10 900 tools/experiments/gpu_ab.sh r4al binorder
