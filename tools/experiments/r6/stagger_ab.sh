#!/bin/bash
# same-box A/B of the staggered slots (env DVBT2LL_STAGGER, read by an experiment build of t2_capi.cpp that was
# reverted: profiles/r6_overlap_trace.txt) on the default bench, two rounds
set -o pipefail
cd "$(dirname "$0")" 2>/dev/null; cd $GRAFT_REPO_ROOT
O=gpurun_out/r6x; mkdir -p $O
for r in 1 2; do
  for st in 0 1; do
    DVBT2LL_STAGGER=$st timeout -k 10 240 python bench.py --no-pmc --no-cpu-baseline --no-latency --no-sc16 --no-blocks --no-mplp --no-host --steps 20 --warmup 3 > $O/b_st${st}_$r.json 2> $O/b_st${st}_$r.err || { tail -5 $O/b_st${st}_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/b_st${st}_$r.json')); print('stagger $st', round(d['value']), round(d['ms_per_step'],3), d['chain']['serial_kernel_ms_per_step'])"
  done
done
