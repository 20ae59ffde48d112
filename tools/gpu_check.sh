#!/bin/bash
# GPU parity tests (all, in one process) then a quick bench without PMC passes / CPU baseline.
# Usage: tools/gpu_check.sh TAG [pytest -k expression].  Each GPU step has its own limit; a failure
# ends the script.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p "$O"
K=()
[ -n "$2" ] && K=(-k "$2")
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  "${K[@]}" > "$O/pytest.log" 2>&1
rc=$?
tail -30 "$O/pytest.log"
[ $rc = 0 ] || exit $rc
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 240 python bench.py --no-pmc --no-cpu-baseline --no-latency --no-sc16 --no-blocks --steps 20 --warmup 3 \
  $BENCH_ARGS > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print({k: round(s['avg_launch_ms'],4) for k,s in d['stages'].items()}, round(d['value']))"
