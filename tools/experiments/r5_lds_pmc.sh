#!/bin/bash
# LDS counters of the LDPC + map kernel for the product and wrong-output probe libraries (exp_ab/lib<v>.so):
# one rocprofv3 --pmc pass each over bench.py --pmc-child.  Usage: tools/experiments/r5_lds_pmc.sh TAG v1 v2 ..
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p "$O"
LIB=gr-dvbt2ll_amd/dvbt2ll/libdvbt2ll_hip.so
cp $LIB exp_ab/libproduct.so
for v in product "$@"; do
  cp exp_ab/lib$v.so $LIB
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES -T -f csv -d $O/pmc_$v -o pmc -- \
    python3 bench.py --pmc-child --no-sc16 --steps 2 --warmup 1 > /dev/null 2> $O/pmc_$v.err
  rc=$?; echo "PMC $v EXIT $rc"; [ $rc = 0 ] || { cp exp_ab/libproduct.so $LIB; exit $rc; }
done
cp exp_ab/libproduct.so $LIB
python3 - "$O" product "$@" <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
for v in sys.argv[2:]:
    acc = collections.defaultdict(list)
    for f in glob.glob("%s/pmc_%s/**/*counter_collection.csv" % (o, v), recursive=True):
        for r in csv.DictReader(open(f)):
            if "ldpc_map" in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(v, {k: "%.4g" % (sum(x) / len(x)) for k, x in sorted(acc.items())})
PY
