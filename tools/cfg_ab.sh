# Same-box A/B of exp_build variants over several configs: VARIANTS="a b" CFGS="cfg2 cfg4:4" bash tools/cfg_ab.sh
# (cfg:S = S independent streams per launch); bench.py without PMC / CPU baseline / secondaries
set -o pipefail
mkdir -p gpurun_out
LIB=gr-dvbt2ll_amd/dvbt2ll/libdvbt2ll_hip.so
cp $LIB /tmp/prod.so
for v in $VARIANTS; do
  cp exp_build/lib$v.so $LIB
  for c in $CFGS; do
    cfg=${c%%:*}; st=1; [ "$c" != "$cfg" ] && st=${c##*:}
    timeout -k 10 120 python bench.py --config $cfg --streams $st --no-pmc --no-cpu-baseline --no-blocks --no-latency --no-sc16 --steps 20 > gpurun_out/cfgab_${v}_$cfg.json 2>/dev/null || { echo "variant $v $c failed"; cp /tmp/prod.so $LIB; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/cfgab_${v}_$cfg.json'));print('variant $v $c', {k:round(x['avg_launch_ms'],4) for k,x in d['stages'].items()}, round(d['value']))"
  done
done
cp /tmp/prod.so $LIB
