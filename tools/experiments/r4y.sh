set -o pipefail
for v in bchks1 bchks2; do
  echo "$v $(timeout -k 10 120 python tools/experiments/lib_iq_hash.py exp_build/lib$v.so)" || exit 1
done &&
NOPROBE=1 timeout -k 10 900 tools/experiments/gpu_ab.sh r4y bchks1 bchks2
