#!/bin/bash
# Kernel trace of the pipelined bench (the default 3 slots / streams) and the overlap attribution
# (tools/overlap_trace.py).  Usage: tools/gpu_overlap.sh TAG [extra bench args]
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/$1; shift; mkdir -p "$O"
timeout -k 10 300 rocprofv3 --kernel-trace -d "$O/otrace" -o otrace -f csv -- \
  python bench.py --no-pmc --no-cpu-baseline --no-latency --no-sc16 --no-blocks --no-host --no-mplp --steps 10 --warmup 2 "$@" \
  > "$O/otrace_bench.json" 2> "$O/otrace.err" || { tail -20 "$O/otrace.err"; exit 1; }
f=$(find "$O/otrace" -name '*kernel_trace.csv' | head -1)
cp "$f" "$O/otrace_kernel_trace.csv"
# the bench runs the pipelined pass (warmup + 10 steps) first, then the serial pass: 3 kernels per step
python tools/overlap_trace.py "$f" --skip 6 --take 30 > "$O/overlap_pipelined.txt" &&
python tools/overlap_trace.py "$f" --skip 36 --take 30 > "$O/overlap_serial.txt" &&
cat "$O/overlap_pipelined.txt" "$O/overlap_serial.txt"
