#!/bin/bash
# One GPU session: parity tests, smoke, bench (PMC passes inside), kernel trace of the bench command.
# Every GPU step has its own time limit; the chain stops at the first failure (no GPU work after it).
# Usage: tools/gpu_session.sh TAG [pytest selection...]   (env: NOBENCH=1, NOTRACE=1, BENCH_ARGS)
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
TAG=${1:-r3}; shift
SEL=("$@"); [ ${#SEL[@]} -gt 0 ] || SEL=(tests)
O=gpurun_out/$TAG
mkdir -p "$O"
rm -f "$O/iq_stats.jsonl"
step() { echo "=== $* ($(date +%T))"; }
step tests && IQ_STATS=$PWD/$O/iq_stats.jsonl timeout -k 10 900 python -u -m pytest "${SEL[@]}" -m gpu -x -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/pytest.log" 2>&1 \
  && tail -3 "$O/pytest.log" \
  && step smoke && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
  && cat "$O/smoke.log" || { rc=$?; tail -30 "$O/pytest.log"; exit $rc; }
[ -n "$NOBENCH" ] && exit 0
step bench && timeout -k 10 900 python -u bench.py $BENCH_ARGS > "$O/bench.json" 2> "$O/bench.err" \
  && cat "$O/bench.json" || { rc=$?; tail -20 "$O/bench.err"; exit $rc; }
[ -n "$NOTRACE" ] && exit 0
step trace && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o trace -f csv -- \
     python bench.py --no-pmc --no-cpu-baseline --no-latency --no-sc16 --no-blocks --no-mplp --no-host --slots 1 --steps 10 --warmup 2 \
     > "$O/trace_bench.json" 2> "$O/trace.err" \
  && echo "=== done ($(date +%T))"
