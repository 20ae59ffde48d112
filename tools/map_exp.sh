set -o pipefail
mkdir -p gpurun_out
LIB=gr-dvbt2ll_amd/dvbt2ll/libdvbt2ll_hip.so
cp $LIB /tmp/prod.so
for v in prod map2; do
  if [ $v != prod ]; then cp exp_build/lib$v.so $LIB; fi
  timeout -k 10 120 python bench.py --no-pmc --no-cpu-baseline --steps 10 > gpurun_out/mapexp_$v.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/mapexp_$v.json'));print('$v', {k:round(v['avg_launch_ms'],4) for k,v in d['stages'].items()})"
done
cp /tmp/prod.so $LIB
