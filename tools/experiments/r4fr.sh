#!/bin/bash
# GPU tests + smoke on the final tree, then frames per step 768 / 1024 / 1280 (two rounds)
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
NOBENCH=1 bash tools/gpu_session.sh r4i4 || exit $?
O=gpurun_out/r4fr; mkdir -p $O
for r in 1 2; do for f in 768 1024 1280; do
  timeout -k 10 240 python bench.py --no-pmc --no-cpu-baseline --no-latency --no-sc16 --no-blocks --no-mplp --steps 10 --warmup 3 --frames $f > $O/b_${f}_$r.json 2> $O/b_${f}_$r.err || { tail -5 $O/b_${f}_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b_${f}_$r.json')); print('frames $f', round(d['value']), round(d['ms_per_step'],3))"
done; done
