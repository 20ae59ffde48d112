# quick GPU iteration + FEC phase probe (experiment build exp_build/libfec1.so)
bash tools/gpu_quick.sh ${1:-q} && cp gr-dvbt2ll_amd/dvbt2ll/libdvbt2ll_hip.so /tmp/p.so && bash tools/fec_phases.sh; cp /tmp/p.so gr-dvbt2ll_amd/dvbt2ll/libdvbt2ll_hip.so
