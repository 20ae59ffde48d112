#!/bin/bash
# Kernel trace of a short bench run: rocprofv3 --kernel-trace --stats (per-kernel averages).
# Usage: tools/gpu_trace.sh TAG [extra bench args]
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/$1; shift; mkdir -p "$O"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o trace -f csv -- \
  python bench.py --no-pmc --no-cpu-baseline --no-latency --no-sc16 --no-blocks --no-host --slots 1 --steps 10 --warmup 2 "$@" \
  > "$O/trace_bench.json" 2> "$O/trace.err" || { tail -20 "$O/trace.err"; exit 1; }
f=$(find "$O/trace" -name '*kernel_stats.csv' | head -1)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    print("%-60s %5s calls  avg %9.1f us  min %9.1f  %5.1f %%" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3,
          float(r["MinNs"]) / 1e3, float(r["Percentage"])))
PY
