set -o pipefail
cp exp_build/libp1.so gr-dvbt2ll_amd/dvbt2ll/libdvbt2ll_hip.so
for g in 256 248 240 224 256; do
  DVBT2LL_O32_GRID=$g timeout -k 10 120 python bench.py --no-pmc --no-cpu-baseline --no-blocks --no-latency --no-sc16 --steps 20 > gpurun_out/og_$g.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/og_$g.json'));print('O32_GRID=$g', {k:round(x['avg_launch_ms'],4) for k,x in d['stages'].items()}, round(d['value']))"
done
for g in 256 248 240 256; do
  DVBT2LL_O32_GRID=224 DVBT2LL_FEC_GRID_CU=$g timeout -k 10 120 python bench.py --no-pmc --no-cpu-baseline --no-blocks --no-latency --no-sc16 --steps 20 > gpurun_out/fg_$g.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/fg_$g.json'));print('FEC_GRID_CU=$g', {k:round(x['avg_launch_ms'],4) for k,x in d['stages'].items()}, round(d['value']))"
done
