#!/bin/bash
# Same-box A/B of experiment libraries: tools/experiments/gpu_ab.sh TAG VARIANT... (product = the
# in-tree library).  Each variant's library replaces the product's for its bench runs only; two rounds.
# Every GPU step has its own limit; the first failure ends the script.
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p "$O"
LIB=gr-dvbt2ll_amd/dvbt2ll/libdvbt2ll_hip.so
E=${EXP:-exp_build}   # variant libraries (exp_build/ is gpurun-ignored: ship them in another directory)
mkdir -p "$E"
cp $LIB $E/libproduct.so
[ -x exp_build/mfma_probe ] && [ -z "$NOPROBE" ] && { timeout -k 10 60 exp_build/mfma_probe "$O/mfma_probe.bin" > "$O/mfma_probe.log" 2>&1 || { cat "$O/mfma_probe.log"; exit 1; }; cat "$O/mfma_probe.log"; }
for round in 1 2; do
  for v in product "$@"; do
    cp $E/lib$v.so $LIB || { echo "missing $E/lib$v.so"; cp $E/libproduct.so $LIB; exit 1; }
    timeout -k 10 240 python bench.py --no-pmc --no-cpu-baseline --no-latency --no-sc16 --no-blocks --no-mplp --steps 20 --warmup 3 $BENCH_ARGS \
      > "$O/b_${v}_$round.json" 2> "$O/b_${v}_$round.err" || { tail -5 "$O/b_${v}_$round.err"; cp $E/libproduct.so $LIB; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/b_${v}_$round.json')); print('$v', {k: round(s['avg_launch_ms'],4) for k,s in d['stages'].items()}, round(d['value']))"
  done
done
cp $E/libproduct.so $LIB
