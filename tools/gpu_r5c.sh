set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5c
timeout -k 10 300 python -u -m pytest tests/test_gpu_host.py tests/test_gpu_chain.py -k "host or tx" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5c/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r5c/pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-pmc --no-cpu-baseline --no-blocks --no-mplp --steps 10 --warmup 2 > gpurun_out/r5c/bench.json 2> gpurun_out/r5c/bench.err || { tail -20 gpurun_out/r5c/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r5c/bench.json')); print(round(d['value']), json.dumps(d.get('host_delivered'), indent=1))"
