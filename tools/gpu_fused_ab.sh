# fused FEC+map A/B on one box: parity tests (default two kernels, then the chain tests fused), then
# bench stages for each setting and config
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/fab_tests.log 2>&1; rc=$?; tail -1 gpurun_out/fab_tests.log; [ $rc = 0 ] || { grep -E "Error|FAIL" gpurun_out/fab_tests.log | head; exit $rc; }
DVBT2LL_CHAIN_FUSED=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/fab_tests_fused.log 2>&1; rc=$?; tail -1 gpurun_out/fab_tests_fused.log; [ $rc = 0 ] || exit $rc
for c in ${CFGS:-cfg3 cfg2 cfg4}; do
  for uf in 0 1; do
    DVBT2LL_CHAIN_FUSED=$uf timeout -k 10 120 python bench.py --config $c --no-pmc --no-cpu-baseline --no-latency --no-sc16 --steps 20 \
      > gpurun_out/fab_${c}_$uf.json 2> gpurun_out/fab_${c}_$uf.err; rc=$?
    [ $rc = 0 ] || { echo "bench $c $uf rc=$rc"; tail -3 gpurun_out/fab_${c}_$uf.err; exit $rc; }
    python -c "import json;d=json.load(open('gpurun_out/fab_${c}_$uf.json'));print('$c fused=$uf', {k:round(v['avg_launch_ms'],4) for k,v in d['stages'].items()}, round(d['value']), 'serial', round(d['serial_1_stream']['value']))"
  done
done
