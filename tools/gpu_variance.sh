#!/bin/bash
# the default bench three times back to back on one box (box-internal spread of the headline), then the GPU suite
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p "$O"
for r in 1 2 3; do
  timeout -k 10 400 python bench.py --no-cpu-baseline > "$O/bench_$r.json" 2> "$O/bench_$r.err" || { tail -5 "$O/bench_$r.err"; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$r.json')); print('run $r', round(d['value']), round(d['ms_per_step'], 3), {k: round(s['avg_launch_ms'], 4) for k, s in d['stages'].items()})"
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > "$O/pytest.log" 2>&1; rc=$?
tail -2 "$O/pytest.log"; exit $rc
