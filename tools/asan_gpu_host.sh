#!/bin/bash
# GPU box: the host-ASan build's drivers against the plain build's (tools/asan_gpu_host.py), time-limited
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/asan_host
timeout -k 10 600 python -u tools/asan_gpu_host.py gpurun_out/asan_host
