# 32K OFDM: parity tests on the product build, same-box A/B of variants, phase probe
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/o32ab_tests.log 2>&1; rc=$?; tail -1 gpurun_out/o32ab_tests.log; [ $rc = 0 ] || exit $rc
LIB=gr-dvbt2ll_amd/dvbt2ll/libdvbt2ll_hip.so
cp $LIB /tmp/prod.so
for v in prod ${VARIANTS:-persist}; do
  [ $v = prod ] || cp exp_build/lib$v.so $LIB
  timeout -k 10 120 python bench.py --no-pmc --no-cpu-baseline --no-latency --no-sc16 --steps 20 > gpurun_out/o32ab_$v.json 2>/dev/null
  rc=$?; [ $rc = 0 ] || { echo "variant $v rc=$rc"; cp /tmp/prod.so $LIB; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/o32ab_$v.json'));print('variant $v', {k:round(v['avg_launch_ms'],4) for k,v in d['stages'].items()}, round(d['value']))"
  cp /tmp/prod.so $LIB
done
cp exp_build/libvar8.so $LIB
timeout -k 10 120 python tools/ofdm_phases.py cfg3 > gpurun_out/o32ab_phases.txt 2>&1; rc=$?
cp /tmp/prod.so $LIB
cat gpurun_out/o32ab_phases.txt
exit $rc
