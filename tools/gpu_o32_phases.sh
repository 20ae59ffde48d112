# phase probe of the 32K OFDM kernel (OFDM_VARIANT=8 build swapped in; wrong output by design)
set -o pipefail
mkdir -p gpurun_out
cp gr-dvbt2ll_amd/dvbt2ll/libdvbt2ll_hip.so /tmp/prod.so
cp exp_build/libvar8.so gr-dvbt2ll_amd/dvbt2ll/libdvbt2ll_hip.so
timeout -k 10 120 python tools/ofdm_phases.py ${1:-cfg3} > gpurun_out/phases_${1:-cfg3}.txt 2>&1; rc=$?
cp /tmp/prod.so gr-dvbt2ll_amd/dvbt2ll/libdvbt2ll_hip.so
cat gpurun_out/phases_${1:-cfg3}.txt
exit $rc
