set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -m gpu -q --tb=short > gpurun_out/t3.log 2>&1; echo "TESTS EXIT $?"; tail -5 gpurun_out/t3.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; echo "SMOKE EXIT $?"; tail -3 gpurun_out/smoke.log
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err; echo "BENCH EXIT $?"; tail -3 gpurun_out/bench.err; cat gpurun_out/bench.json
