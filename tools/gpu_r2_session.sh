#!/bin/bash
# One GPU session (round 2): parity tests, smoke, FETCH/WRITE_SIZE calibration, bench, kernel trace.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
TAG=${1:-r2a}
O=gpurun_out/$TAG
mkdir -p "$O"
rm -f "$O/iq_stats.jsonl"
step() { echo "=== $* ($(date +%T))"; }
step tests && IQ_STATS=$PWD/$O/iq_stats.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -x -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/pytest.log" 2>&1 \
  && tail -3 "$O/pytest.log" \
  && step smoke && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
  && cat "$O/smoke.log" \
  && if [ -n "$CALIB" ]; then step calib && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -T -d "$O/calib_fetch" -o calib -- ./tools/fetch_calib > /dev/null 2>&1 \
  && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -T -d "$O/calib_write" -o calib -- ./tools/fetch_calib > /dev/null 2>&1 \
  && python tools/fetch_calib.py "$O/calib_fetch" "$O/calib_write" > "$O/r2_fetch_calib.json" \
  && cp "$O/r2_fetch_calib.json" profiles/r2_fetch_calib.json && cat "$O/r2_fetch_calib.json"; fi \
  && step bench && timeout -k 10 900 python -u bench.py > "$O/bench.json" 2> "$O/bench.err" \
  && cat "$O/bench.json" \
  && step trace && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o trace -f csv -- \
       python bench.py --no-pmc --no-cpu-baseline --no-latency --no-sc16 --no-blocks --slots 1 --steps 10 --warmup 2 \
       > "$O/trace_bench.json" 2> "$O/trace.err" \
  && echo "=== done ($(date +%T))"
rc=$?
[ $rc -eq 0 ] || exit $rc
# multi-stream batches (BASELINE cfg4 x4, cfg5 x8 streams in one launch), when asked for
if [ -n "$STREAMS" ]; then
  step streams && timeout -k 10 300 python -u bench.py --config cfg4 --streams 4 --no-pmc --no-cpu-baseline --no-sc16 \
       > "$O/bench_cfg4_x4.json" 2> "$O/bench_cfg4_x4.err" \
    && timeout -k 10 300 python -u bench.py --config cfg5 --streams 8 --no-pmc --no-cpu-baseline --no-sc16 \
       > "$O/bench_cfg5_x8.json" 2> "$O/bench_cfg5_x8.err" && echo "=== streams done"
fi
# raw PMC passes of the bench child kept for inspection, when asked for
if [ -n "$PMCDBG" ]; then
  step pmcdbg && for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c -T -f csv \
      -d "$O/pmc_$c" -o pmc -- python bench.py --pmc-child --steps 2 --warmup 1 > "$O/pmc_$c.log" 2>&1 || exit 1
  done && echo "=== pmcdbg done"
fi
