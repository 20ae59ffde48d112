set -o pipefail
for v in mapp2 mapp3; do
  echo "$v $(timeout -k 10 120 python tools/experiments/lib_iq_hash.py exp_build/lib$v.so)" || exit 1
done &&
BENCH_ARGS="--frames 192" NOPROBE=1 timeout -k 10 900 tools/experiments/gpu_ab.sh r4ac mapp2 mapp3
