set -o pipefail
# ldpc_map_kernel r-grouped block order (XCD x: an eighth of the block indices of each 8 frames) against the
# product's frame-major order; IQ hash equality first
h=$(timeout -k 10 120 python tools/experiments/lib_iq_hash.py exp_build/libbase.so) && echo "base $h" &&
h1=$(timeout -k 10 120 python tools/experiments/lib_iq_hash.py exp_build/librgrp.so) && echo "rgrp $h1" &&
[ "$h" = "$h1" ] &&
NOPROBE=1 timeout -k 10 900 tools/experiments/gpu_ab.sh r4ao rgrp
