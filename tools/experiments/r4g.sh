set -o pipefail
mkdir -p gpurun_out/r4g
for v in r4base xr; do
  echo "$v $(timeout -k 10 120 python tools/experiments/lib_iq_hash.py exp_build/lib$v.so)" || exit 1
done &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -x -q -k "cfg3 or cfg2 or cfg5 or 32k" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4g/chain.log 2>&1 && tail -2 gpurun_out/r4g/chain.log &&
NOPROBE=1 timeout -k 10 900 tools/experiments/gpu_ab.sh r4g r4base xrplain
