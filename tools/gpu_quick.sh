# Quick GPU iteration: parity tests, then a short bench (no PMC passes, no CPU baseline).
# Each GPU step has its own time limit; any failure ends the script (no further GPU work).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-q}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --tb=short -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
rc=$?
tail -25 gpurun_out/tests_$TAG.log
echo "STEP tests EXIT $rc"
[ $rc = 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-pmc --no-cpu-baseline $BENCH_ARGS > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?
echo "STEP bench EXIT $rc"
[ $rc = 0 ] || { tail -5 gpurun_out/bench_$TAG.err; exit $rc; }
python - <<EOF
import json; d = json.load(open("gpurun_out/bench_$TAG.json"))
print("value %.0f Msps  ms/step %.3f  serial %.0f  sc16 %.0f" % (d["value"], d["ms_per_step"], d["serial_1_stream"]["value"], d.get("iq_sc16_x0.2", {}).get("value", 0)))
for k, v in d["stages"].items(): print("  %-5s %.4f ms  %.0f GB/s" % (k, v["avg_launch_ms"], v["achieved_GBs"]))
print("latency", d["latency_1_frame"])
EOF
