#!/bin/bash
# frames-per-step and slot-count sweep of the default bench (round-6 kernels): one JSON line each under gpurun_out/$1
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/$1; mkdir -p "$O"
run() {
  timeout -k 10 300 python bench.py --no-pmc --no-cpu-baseline --no-latency --no-sc16 --no-blocks --no-mplp --no-host --steps 20 --warmup 3 "$@" \
    > "$O/b$(echo "$@" | tr ' ' '_').json" 2> "$O/b.err" || { tail -5 "$O/b.err"; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/b$(echo "$@" | tr ' ' '_').json')); print('$*', round(d['value']), round(d['ms_per_step'], 3))"
}
for f in 192 384 768 1024 1280 1359; do run --frames $f; done
for s in 1 2 4; do run --slots $s; done
