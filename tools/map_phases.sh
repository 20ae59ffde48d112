set -o pipefail
mkdir -p gpurun_out
make -s -C gr-dvbt2ll_amd/csrc probe
cp exp_build/libmap1.so gr-dvbt2ll_amd/dvbt2ll/libdvbt2ll_hip.so
timeout -k 10 120 python tools/map_phases.py cfg3 > gpurun_out/map_phases_cfg3.txt 2>&1; echo rc=$?
cat gpurun_out/map_phases_cfg3.txt
