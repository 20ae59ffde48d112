set -o pipefail
# map_cells: the column windows' bytes assembled with byte permutes (perm); 192 frames per step
h=$(timeout -k 10 120 python tools/experiments/lib_iq_hash.py exp_build/libperm.so) && echo "perm $h" &&
echo "product $(timeout -k 10 120 python tools/experiments/lib_iq_hash.py gr-dvbt2ll_amd/dvbt2ll/libdvbt2ll_hip.so)" &&
BENCH_ARGS="--frames 192" NOPROBE=1 timeout -k 10 900 tools/experiments/gpu_ab.sh r4aj perm
