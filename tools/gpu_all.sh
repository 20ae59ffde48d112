# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel trace + PMC passes.
# Each GPU step has its own time limit; a crash/abort/timeout ends the script (no further GPU work).
set -o pipefail
exec 3>&1
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
TAG=${1:-run}
step() {  # step <name> <seconds> <cmd...>; stops the script on a crash-class exit code
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@"; local rc=$?
  echo "STEP $name EXIT $rc" >&3
  case $rc in 124|134|137|139) echo "STOP after $name" >&3; exit $rc;; esac
  return 0
}
step tests 600 python -m pytest tests -m gpu -q --tb=short -x -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1
tail -5 gpurun_out/tests_$TAG.log
step smoke 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
tail -2 gpurun_out/smoke_$TAG.log
step bench 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
cat gpurun_out/bench_$TAG.json
step trace 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/prof/trace_$TAG -o bench -- python3 bench.py --steps 10 --warmup 2 --no-pmc --no-cpu-baseline --no-sc16 --no-latency --slots 1 > gpurun_out/prof/trace_$TAG.json 2> gpurun_out/prof/trace_$TAG.err
if [ "${PMC:-1}" = 1 ]; then
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE"; do
  t=$(echo $set | tr ' ' '_' | cut -c1-40)
  step pmc_$t 240 rocprofv3 --pmc $set -T -f csv -d gpurun_out/prof/pmc_${TAG}_$t -o pmc -- python3 bench.py --pmc-child --no-sc16 --steps 2 --warmup 1 > /dev/null 2> gpurun_out/prof/pmc_${TAG}_$t.err
done
fi
echo ALLDONE
