# PMC counter passes over bench.py --pmc-child (one rocprofv3 run per counter set, each time-limited)
#   [PMC_ARGS="--config cfg4"] bash tools/gpu_pmc.sh <tag> "<set1>" "<set2>" ...
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
TAG=$1; shift
for set in "$@"; do
  t=$(echo $set | tr ' ' '_' | cut -c1-40)
  timeout -s KILL 120 rocprofv3 --pmc $set -T -f csv -d gpurun_out/prof/pmc_${TAG}_$t -o pmc -- python3 bench.py --pmc-child $PMC_ARGS --no-sc16 --steps 2 --warmup 1 > /dev/null 2> gpurun_out/prof/pmc_${TAG}_$t.err
  rc=$?; echo "PMC $t EXIT $rc"
  [ $rc = 0 ] || exit $rc
done
python3 - "$TAG" <<'PY'
import csv, glob, sys, collections
tag = sys.argv[1]
acc = collections.defaultdict(list)
for f in glob.glob("gpurun_out/prof/pmc_%s_*/**/*counter_collection.csv" % tag, recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][-24:]
        acc[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    print("%-26s %-28s %.4g" % (k, c, sum(v) / len(v)))
PY
