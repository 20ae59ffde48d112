set -o pipefail
# fused LDPC + map (product) against HEAD (base) at the bench's default 768 frames per step
NOPROBE=1 timeout -k 10 1000 tools/experiments/gpu_ab.sh r4af base
