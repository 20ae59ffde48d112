set -o pipefail
for v in x1w128b; do
  echo "$v $(timeout -k 10 120 python tools/experiments/lib_iq_hash.py exp_build/lib$v.so)" || exit 1
done &&
echo "product $(timeout -k 10 120 python tools/experiments/lib_iq_hash.py gr-dvbt2ll_amd/dvbt2ll/libdvbt2ll_hip.so)" &&
BENCH_ARGS="--frames 192" NOPROBE=1 timeout -k 10 900 tools/experiments/gpu_ab.sh r4ad x1w128b
