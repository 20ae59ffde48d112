# r5d: the host ASan run with the multi-PLP cases (outputs in /tmp, only the log comes back)
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5d
timeout -k 10 600 python -u tools/asan_gpu_host.py /tmp/asan_host > gpurun_out/r5d/asan.txt 2>&1
rc=$?; cp /tmp/asan_host/asan_host.log gpurun_out/r5d/asan_host.log 2>/dev/null; tail -5 gpurun_out/r5d/asan.txt; exit $rc
