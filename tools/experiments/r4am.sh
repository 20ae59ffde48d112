set -o pipefail
# ldpc_map_kernel with the frame held as big-endian words (the codeword's head in place; only the LDPC
# parity words are built), product against HEAD (base); 192 frames per step
h=$(timeout -k 10 120 python tools/experiments/lib_iq_hash.py exp_build/libbase.so) && echo "base $h" &&
h=$(timeout -k 10 120 python tools/experiments/lib_iq_hash.py gr-dvbt2ll_amd/dvbt2ll/libdvbt2ll_hip.so) && echo "product $h" &&
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "codewords or chain_iq or mplp" > gpurun_out/r4am_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4am_tests.log; [ $rc -eq 0 ] &&
BENCH_ARGS="--frames 192" NOPROBE=1 timeout -k 10 900 tools/experiments/gpu_ab.sh r4am base
