#!/bin/bash
# kernel trace of the one-frame latency calls (direct, then hipGraph mode): gaps between a call's kernels
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4gl; mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace -d $O/trace -o trace -f csv -- \
  python bench.py --no-pmc --no-cpu-baseline --no-sc16 --no-blocks --no-mplp --steps 1 --warmup 1 --frames 8 \
  > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
python -c "import json; print(json.load(open('$O/b.json'))['latency_1_frame'])"
