set -o pipefail
# 32K OFDM frame-fast workgroups in plain dispatch order against the product's XCD-major order; IQ hash first
h=$(timeout -k 10 120 python tools/experiments/lib_iq_hash.py exp_build/libbase.so) && echo "base $h" &&
h1=$(timeout -k 10 120 python tools/experiments/lib_iq_hash.py exp_build/libplain.so) && echo "plain $h1" &&
[ "$h" = "$h1" ] &&
NOPROBE=1 timeout -k 10 900 tools/experiments/gpu_ab.sh r4aq plain
