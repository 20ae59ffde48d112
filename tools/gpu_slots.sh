# slots experiment: new chain tests, then the bench at 1 and 2 slots (no PMC / CPU baseline)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-sl}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --tb=short -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
rc=$?; tail -5 gpurun_out/tests_$TAG.log; echo "STEP tests EXIT $rc"; [ $rc = 0 ] || exit $rc
for S in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-pmc --no-cpu-baseline --slots $S > gpurun_out/bench_${TAG}_$S.json 2> gpurun_out/bench_${TAG}_$S.err
  rc=$?; echo "STEP bench slots=$S EXIT $rc"; [ $rc = 0 ] || { tail -5 gpurun_out/bench_${TAG}_$S.err; exit $rc; }
  python - <<PY
import json; d = json.load(open("gpurun_out/bench_${TAG}_$S.json"))
print("slots $S value %.0f Msps  ms/step %.3f  sc16 %.0f" % (d["value"], d["ms_per_step"], d["iq_sc16_x0.2"]["value"]))
for k, v in d["stages"].items(): print("  %-5s %.4f ms  %.0f GB/s" % (k, v["avg_launch_ms"], v["achieved_GBs"]))
PY
done
