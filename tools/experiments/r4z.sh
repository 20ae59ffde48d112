set -o pipefail
mkdir -p gpurun_out/r4z
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4z/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r4z/pytest.log; [ $rc = 0 ] || exit $rc
for fr in 192 384 768; do
  timeout -k 10 300 python bench.py --no-pmc --no-cpu-baseline --no-latency --no-sc16 --no-blocks --no-mplp --steps 20 --warmup 3 --frames $fr > gpurun_out/r4z/b_$fr.json 2> gpurun_out/r4z/b_$fr.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/r4z/b_$fr.json')); print('frames $fr', round(d['value']), round(d['ms_per_step'],4), {k: round(s['avg_launch_ms'],4) for k,s in d['stages'].items()})"
done
