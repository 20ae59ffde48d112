set -o pipefail
mkdir -p gpurun_out/r4l
timeout -k 10 240 tools/store_rate > gpurun_out/r4l/store_rate.jsonl; rc=$?; cat gpurun_out/r4l/store_rate.jsonl; exit $rc
