# bench.py on every config (cfg1-cfg5), no PMC / CPU baseline / per-block / 2-PLP lines: one JSON line per
# config (BENCH_ARGS: extra bench.py arguments, e.g. --frames 192); TAG names the output files
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-cfgs}
for c in cfg1 cfg2 cfg3 cfg4 cfg5; do
  timeout -k 10 180 python bench.py --config $c --steps 20 --warmup 3 --no-pmc --no-cpu-baseline --no-sc16 --no-blocks --no-mplp $BENCH_ARGS > gpurun_out/${TAG}_$c.json 2> gpurun_out/${TAG}_$c.err
  rc=$?; echo "config $c rc=$rc"; [ $rc = 0 ] || { tail -3 gpurun_out/${TAG}_$c.err; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_$c.json'));print('$c', round(d['value']), 'Msps x%.0f RT' % d['x_realtime'], round(d['fec_blocks_per_sec']), 'FEC/s', {k:round(v['avg_launch_ms'],4) for k,v in d['stages'].items()}, 'frac %.2f' % d['roofline']['frac'], 'lat %.3f ms' % d['latency_1_frame']['median_ms'])"
done
