set -o pipefail
# phase costs of ldpc_map_kernel by wrong-output subtraction (no TI store / no column twist + demux /
# no LDPC parity / no codeword words), 192 frames per step
BENCH_ARGS="--frames 192" NOPROBE=1 timeout -k 10 1000 tools/experiments/gpu_ab.sh r4ag nostore nocells noldpc nowords
