# bench.py on every config (cfg1-cfg5), no PMC / CPU baseline: one JSON line per config
set -o pipefail
mkdir -p gpurun_out
for c in cfg1 cfg2 cfg3 cfg4 cfg5; do
  timeout -k 10 120 python bench.py --config $c --steps 20 --warmup 3 --no-pmc --no-cpu-baseline --no-sc16 > gpurun_out/cfgs_$c.json 2> gpurun_out/cfgs_$c.err
  rc=$?; echo "config $c rc=$rc"; [ $rc = 0 ] || { tail -3 gpurun_out/cfgs_$c.err; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/cfgs_$c.json'));print('$c', round(d['value']), 'Msps x%.0f RT' % d['x_realtime'], round(d['fec_blocks_per_sec']), 'FEC/s', {k:round(v['avg_launch_ms'],4) for k,v in d['stages'].items()}, 'frac %.2f' % d['roofline']['frac'], 'lat %.3f ms' % d['latency_1_frame']['median_ms'])"
done
