#!/bin/bash
# bench.py on every config (cfg1-cfg5) WITH its rocprofv3 PMC passes (FETCH_SIZE / WRITE_SIZE / SQ instruction
# counts per kernel), no CPU baseline / per-block / 2-PLP lines; one JSON line per config under gpurun_out/
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-cfgpmc}
export TMPDIR=/tmp
for c in cfg1 cfg2 cfg3 cfg4 cfg5; do
  timeout -k 10 420 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-sc16 --no-blocks --no-mplp --no-host \
    > gpurun_out/${TAG}_$c.json 2> gpurun_out/${TAG}_$c.err
  rc=$?; echo "config $c rc=$rc"; [ $rc = 0 ] || { tail -3 gpurun_out/${TAG}_$c.err; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_$c.json'));print('$c', round(d['value']), {k:(round(v['avg_launch_ms'],4), round(v.get('traffic_over_min') or 0,3)) for k,v in d['rooflines'].items()}, 'chain mand %.3f pmc %.3f' % (d['chain']['mandatory_bytes_frac'], d['chain'].get('pmc_bytes_frac') or 0))"
done
