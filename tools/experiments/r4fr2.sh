#!/bin/bash
# frames per step sweep (pipelined bench step, serial per-stage times)
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r4fr2; mkdir -p $O
for f in 768 896 1152 1280 1344 640 1280 768; do
  timeout -k 10 240 python bench.py --no-pmc --no-cpu-baseline --no-latency --no-sc16 --no-blocks --no-mplp --steps 10 --warmup 3 --frames $f > $O/b_$f.json 2> $O/b_$f.err || { tail -5 $O/b_$f.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b_$f.json')); print('frames $f', round(d['value']), round(d['ms_per_step'],3), {k: round(v['avg_launch_ms']*192/$f,4) for k,v in d['stages'].items()})"
done
