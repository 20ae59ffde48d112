set -o pipefail
mkdir -p gpurun_out/r4u
for sl in 1 2 3 4; do
  timeout -k 10 240 python bench.py --no-pmc --no-cpu-baseline --no-latency --no-sc16 --no-blocks --no-mplp --steps 20 --warmup 3 --slots $sl > gpurun_out/r4u/b_$sl.json 2> gpurun_out/r4u/b_$sl.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/r4u/b_$sl.json')); print('slots $sl', round(d['value']), round(d['ms_per_step'],4))"
done
