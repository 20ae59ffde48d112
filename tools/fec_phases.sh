set -o pipefail
mkdir -p gpurun_out
cp exp_build/lib${FECV:-fec1}.so gr-dvbt2ll_amd/dvbt2ll/libdvbt2ll_hip.so
timeout -k 10 120 python tools/fec_phases.py cfg3 > gpurun_out/fec_phases_cfg3.txt 2>&1; echo rc=$?
cat gpurun_out/fec_phases_cfg3.txt
