#!/bin/bash
# frames per step x slots / streams (CASES: ";"-separated bench arguments), two rounds
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r4fr3; mkdir -p $O
IFS=";" read -ra CL <<< "${CASES:-"--frames 1280 --slots 2;--frames 1280 --slots 3;--frames 1359 --slots 2"}"
for r in 1 2; do for a in "${CL[@]}"; do
  t=$(echo $a | tr -d ' -')_$r
  timeout -k 10 240 python bench.py --no-pmc --no-cpu-baseline --no-latency --no-sc16 --no-blocks --no-mplp --steps 10 --warmup 3 $a > $O/b_$t.json 2> $O/b_$t.err || { tail -5 $O/b_$t.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b_$t.json')); print('$a', round(d['value']), round(d['ms_per_step'],3))"
done; done
