set -o pipefail
mkdir -p gpurun_out
for f in ${FRAMES:-16 32 64 128}; do
  timeout -k 10 200 python bench.py --no-pmc --no-cpu-baseline --frames $f --steps 10 > gpurun_out/frames_$f.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/frames_$f.json'));print('frames $f', round(d['value']), {k:round(v['avg_launch_ms']/$f*1000,2) for k,v in d['stages'].items()}, 'us/frame')"
done
