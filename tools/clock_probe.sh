# Effective shader clock per kernel (GRBM_GUI_ACTIVE / 8 XCDs / kernel time) for exp_build variants:
#   VARIANTS="sc0 sc1" bash tools/clock_probe.sh
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
LIB=gr-dvbt2ll_amd/dvbt2ll/libdvbt2ll_hip.so
cp $LIB /tmp/prod.so
for v in $VARIANTS; do
  cp exp_build/lib$v.so $LIB
  rm -rf gpurun_out/prof/clk_$v
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -f csv -d gpurun_out/prof/clk_$v -o clk -- python3 bench.py --pmc-child --no-sc16 --steps 4 --warmup 2 > /dev/null 2> gpurun_out/prof/clk_$v.err
  rc=$?; echo "variant $v rc=$rc"; [ $rc = 0 ] || break
  python3 - gpurun_out/prof/clk_$v $v <<'PY'
import csv, glob, sys, collections
d, v = sys.argv[1], sys.argv[2]
dur = collections.defaultdict(list)
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        dur[r["Kernel_Name"].split("(")[0][-20:]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
cnt = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        cnt[r["Kernel_Name"].split("(")[0][-20:]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in cnt.items():
    if k not in dur or "GRBM_GUI_ACTIVE" not in c: continue
    g = sum(c["GRBM_GUI_ACTIVE"]) / len(c["GRBM_GUI_ACTIVE"]); t = sum(dur[k]) / len(dur[k])
    gc = sum(c["GRBM_COUNT"]) / len(c["GRBM_COUNT"]) if "GRBM_COUNT" in c else 0
    print("%s %-20s %.1f us  GUI_ACTIVE/8/t = %.2f GHz  COUNT/8/t = %.2f GHz" % (v, k, t * 1e6, g / 8 / t * 1e-9, gc / 8 / t * 1e-9))
PY
done
cp /tmp/prod.so $LIB
