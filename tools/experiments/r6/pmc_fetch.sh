#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the chain's kernels for each library given (exp_ab/lib<name>.so swapped in)
set -o pipefail
cd "$(dirname "$0")/../../.."
cp gr-dvbt2ll_amd/dvbt2ll/libdvbt2ll_hip.so /tmp/prod.so
rc=0
for v in "$@"; do
  cp exp_ab/lib$v.so gr-dvbt2ll_amd/dvbt2ll/libdvbt2ll_hip.so
  bash tools/gpu_pmc.sh f$v "FETCH_SIZE" "WRITE_SIZE" > gpurun_out/pmcf_$v.txt 2>&1 || { rc=$?; break; }
  grep -E "FETCH|WRITE" gpurun_out/pmcf_$v.txt | sed "s/^/$v /"
done
cp /tmp/prod.so gr-dvbt2ll_amd/dvbt2ll/libdvbt2ll_hip.so
exit $rc
