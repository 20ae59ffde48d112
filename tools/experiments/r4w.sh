set -o pipefail
mkdir -p gpurun_out/r4w
for v in head product; do
  L=exp_build/lib$v.so; [ $v = product ] && L=gr-dvbt2ll_amd/dvbt2ll/libdvbt2ll_hip.so
  echo "$v $(timeout -k 10 120 python tools/experiments/lib_iq_hash.py $L)" || exit 1
done &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4w/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r4w/pytest.log; [ $rc = 0 ] || exit $rc
NOPROBE=1 timeout -k 10 900 tools/experiments/gpu_ab.sh r4w head
