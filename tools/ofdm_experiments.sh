# Swap experimental builds of the kernel library (exp_build/lib<name>.so, tools/build_variant.sh)
# into this (scratch) snapshot and time the chain stages with bench.py for each.
#   VARIANTS="st0 st1" bash tools/ofdm_experiments.sh
set -o pipefail
mkdir -p gpurun_out
LIB=gr-dvbt2ll_amd/dvbt2ll/libdvbt2ll_hip.so
cp $LIB /tmp/prod.so
for v in ${VARIANTS:-st0}; do
  cp exp_build/lib$v.so $LIB
  timeout -k 10 120 python bench.py --no-pmc --no-cpu-baseline --steps 20 > gpurun_out/exp_$v.json 2>/dev/null
  rc=$?; echo "variant $v rc=$rc"
  case $rc in 0) ;; *) break;; esac
  python -c "import json;d=json.load(open('gpurun_out/exp_$v.json'));print('variant $v', {k:round(v['avg_launch_ms'],4) for k,v in d['stages'].items()}, round(d['value']))"
done
cp /tmp/prod.so $LIB
