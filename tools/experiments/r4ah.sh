set -o pipefail
# ldpc_map_kernel: branchless index-pair reads in the TI quad store (qbl), column windows read four at a
# time in map_cells (cbat4), both (qc4); 192 frames per step
for v in qbl cbat4 qc4; do
  echo "$v $(timeout -k 10 120 python tools/experiments/lib_iq_hash.py exp_build/lib$v.so)" || exit 1
done &&
echo "product $(timeout -k 10 120 python tools/experiments/lib_iq_hash.py gr-dvbt2ll_amd/dvbt2ll/libdvbt2ll_hip.so)" &&
BENCH_ARGS="--frames 192" NOPROBE=1 timeout -k 10 900 tools/experiments/gpu_ab.sh r4ah qbl cbat4 qc4
