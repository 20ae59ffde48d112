# four-step 32K prototype timing (tools/experiments/fourstep_probe.hip), several chunk sizes
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r5fs
for c in 480 240 960 1920; do
  timeout -k 10 120 ./exp_build/fourstep_probe 76800 $c 2 >> gpurun_out/r5fs/probe.jsonl 2>&1 || exit 1
done
cat gpurun_out/r5fs/probe.jsonl
