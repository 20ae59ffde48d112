set -o pipefail
mkdir -p gpurun_out/r4h
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4h/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r4h/pytest.log; [ $rc = 0 ] || exit $rc
NOPROBE=1 timeout -k 10 900 tools/experiments/gpu_ab.sh r4h r4base ldpc1
