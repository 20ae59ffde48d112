set -o pipefail
mkdir -p gpurun_out/r4f
timeout -k 10 120 tools/store_rate > gpurun_out/r4f/store_rate.jsonl && cat gpurun_out/r4f/store_rate.jsonl &&
for v in product o32pers o32pair o32plain; do
  L=gr-dvbt2ll_amd/dvbt2ll/libdvbt2ll_hip.so; [ $v = product ] || L=exp_build/lib$v.so
  echo "$v $(timeout -k 10 120 python tools/experiments/lib_iq_hash.py $L)" || exit 1
done &&
timeout -k 10 900 tools/experiments/gpu_ab.sh r4f o32pers o32pair o32plain
