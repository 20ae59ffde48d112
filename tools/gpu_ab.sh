set -o pipefail
bash tools/gpu_quick.sh zr || exit $?
VARIANTS="base zr base zr" bash tools/ofdm_experiments.sh
