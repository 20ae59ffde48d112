set -o pipefail
mkdir -p gpurun_out/r4o
timeout -k 10 300 tools/store_rate > gpurun_out/r4o/store_rate.jsonl; rc=$?; grep duty gpurun_out/r4o/store_rate.jsonl; exit $rc
