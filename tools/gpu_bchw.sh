# FEC BCH wave-count A/B on one box: parity of the FEC paths for each setting, then the bench stages.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in ${WAVES:-1 2 4}; do
  DVBT2LL_FEC_BCH_WAVES=$w timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread -k "bbheader or ldpc or chain_cells or chain_iq" > gpurun_out/bchw_tests_$w.log 2>&1
  rc=$?; echo "waves $w tests rc=$rc $(tail -1 gpurun_out/bchw_tests_$w.log)"
  [ $rc = 0 ] || exit $rc
done
for w in ${WAVES:-1 2 4}; do
  DVBT2LL_FEC_BCH_WAVES=$w timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-pmc --no-cpu-baseline \
    --no-latency --no-sc16 $BENCH_ARGS > gpurun_out/bchw_$w.json 2> gpurun_out/bchw_$w.err
  rc=$?; [ $rc = 0 ] || { echo "bench rc=$rc"; tail -3 gpurun_out/bchw_$w.err; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/bchw_$w.json'));print('waves $w', {k:round(v['avg_launch_ms'],4) for k,v in d['stages'].items()}, round(d['value']))"
done
