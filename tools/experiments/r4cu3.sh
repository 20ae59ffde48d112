#!/bin/bash
# kernel trace of the bench with the CU split (queue ids and start / end times of every dispatch)
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4cu3; mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace -d $O/trace -o trace -f csv -- \
  python bench.py --no-pmc --no-cpu-baseline --no-latency --no-sc16 --no-blocks --no-mplp --steps 6 --warmup 2 --cu-split 160 \
  > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
cat $O/b.json | head -c 300; echo
find $O/trace -name "*.csv" | head
