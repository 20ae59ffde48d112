set -o pipefail
mkdir -p gpurun_out/r4ae
echo "base $(timeout -k 10 120 python tools/experiments/lib_iq_hash.py exp_build/libbase.so)" &&
echo "product $(timeout -k 10 120 python tools/experiments/lib_iq_hash.py gr-dvbt2ll_amd/dvbt2ll/libdvbt2ll_hip.so)" &&
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "chain or mplp or bench_shapes or golden or adapter or edges" > gpurun_out/r4ae/tests.log 2>&1; rc=$?; tail -3 gpurun_out/r4ae/tests.log; [ $rc -eq 0 ] &&
BENCH_ARGS="--frames 192" NOPROBE=1 timeout -k 10 900 tools/experiments/gpu_ab.sh r4ae base
