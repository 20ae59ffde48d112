set -o pipefail
NOPROBE=1 timeout -k 10 900 tools/experiments/gpu_ab.sh r4v mnoti2 mnol1 mnoload mnocil
