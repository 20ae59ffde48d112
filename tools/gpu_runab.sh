#!/bin/bash
# A/B of an integer experiment knob over configs: for each VALUE in $VALS and config in $CFGS, one
# short bench.py line with $KNOB=VALUE (stage times only).  Usage: KNOB=.. VALS=".." CFGS=".." tools/gpu_runab.sh TAG
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/$1; mkdir -p "$O"
for c in $CFGS; do
  for v in $VALS; do
    export "$KNOB=$v"
    timeout -k 10 180 python bench.py --config $c --steps 20 --warmup 3 --no-pmc --no-cpu-baseline --no-sc16 --no-blocks \
      --no-mplp --no-host --no-latency $BENCH_ARGS > "$O/${c}_$v.json" 2> "$O/${c}_$v.err" || { tail -5 "$O/${c}_$v.err"; exit 1; }
    python -c "import json;d=json.load(open('$O/${c}_$v.json'));print('$c $KNOB=$v', round(d['value']), {k:round(s['avg_launch_ms'],4) for k,s in d['stages'].items()}, 'frac %.3f' % d['roofline']['frac'])"
  done
done
