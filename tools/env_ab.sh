# same-box A/B of an environment knob: ENVVAR=name VALUES="0 1 0 1" bash tools/env_ab.sh
set -o pipefail
mkdir -p gpurun_out
for v in $VALUES; do
  env $ENVVAR=$v timeout -k 10 120 python bench.py --no-pmc --no-cpu-baseline --no-blocks --no-latency --steps 20 > gpurun_out/envab_$v.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/envab_$v.json'));print('$ENVVAR=$v', {k:round(x['avg_launch_ms'],4) for k,x in d['stages'].items()}, round(d['value']))"
done
