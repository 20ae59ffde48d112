# parity tests on the product build, then same-box A/B timing of exp_build variants ($VARIANTS)
set -o pipefail
bash tools/gpu_quick.sh ${TAG:-ab} || exit $?
VARIANTS="$VARIANTS" bash tools/ofdm_experiments.sh
