set -o pipefail
# 32K OFDM workgroup order: symbol-fast (XCD-major runs of frames; and without XCD-major) against the
# product's frame-fast order; IQ hash equality first
h=$(timeout -k 10 120 python tools/experiments/lib_iq_hash.py exp_build/libbase.so) && echo "base $h" &&
h1=$(timeout -k 10 120 python tools/experiments/lib_iq_hash.py exp_build/libsfast.so) && echo "sfast $h1" &&
h2=$(timeout -k 10 120 python tools/experiments/lib_iq_hash.py exp_build/libsfastrr.so) && echo "sfastrr $h2" &&
[ "$h" = "$h1" ] && [ "$h" = "$h2" ] &&
NOPROBE=1 timeout -k 10 900 tools/experiments/gpu_ab.sh r4an sfast sfastrr
