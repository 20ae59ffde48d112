set -o pipefail
# nontemporal loads of read-once inputs: OFDM index-pair octets (ntp), LDPC + map BBFRAME units (ntb);
# IQ hash equality first
h=$(timeout -k 10 120 python tools/experiments/lib_iq_hash.py exp_build/libbase.so) && echo "base $h" &&
h1=$(timeout -k 10 120 python tools/experiments/lib_iq_hash.py exp_build/libntp.so) && echo "ntp $h1" &&
h2=$(timeout -k 10 120 python tools/experiments/lib_iq_hash.py exp_build/libntb.so) && echo "ntb $h2" &&
[ "$h" = "$h1" ] && [ "$h" = "$h2" ] &&
NOPROBE=1 timeout -k 10 900 tools/experiments/gpu_ab.sh r4ap ntp ntb
