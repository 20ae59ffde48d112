set -o pipefail
cp gr-dvbt2ll_amd/dvbt2ll/libdvbt2ll_hip.so /tmp/prod.so
bash tools/ofdm_phases.sh && bash tools/fec_phases.sh && bash tools/map_phases.sh
cp /tmp/prod.so gr-dvbt2ll_amd/dvbt2ll/libdvbt2ll_hip.so
