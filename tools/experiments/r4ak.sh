set -o pipefail
# ldpc_map_kernel occupancy / TI-store batch: launch bounds 6 workgroups per CU (lb6), MQ = 6 quad rounds
# per batch (mq6), both 6 per CU and MQ = 12 (lb6mq12); 192 frames per step
for v in lb6 mq6 lb6mq12; do
  h=$(timeout -k 10 120 python tools/experiments/lib_iq_hash.py exp_build/lib$v.so) && echo "$v $h" || exit 1
done &&
BENCH_ARGS="--frames 192" NOPROBE=1 timeout -k 10 900 tools/experiments/gpu_ab.sh r4ak lb6 mq6 lb6mq12
