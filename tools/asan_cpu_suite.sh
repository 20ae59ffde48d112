#!/bin/bash
# The CPU test suite's oracle and planner tests against ASan + UBSan builds of the oracle
# (oracle/_build/asan) and of the planner probe (gr-dvbt2ll_amd/csrc/_obj/asan): SURVEY 5's
# "oracle harness under ASan".  Python itself is not instrumented, so the sanitizer runtimes are
# preloaded.  Usage: tools/asan_cpu_suite.sh [pytest args]  (default: the oracle / plan / golden tests)
set -e -o pipefail
cd "$(dirname "$0")/.."
make -s -C oracle asan
make -s -C gr-dvbt2ll_amd/csrc asan
export DVBT2LL_SANITIZED=1
# the sanitizer runtimes first, anything already preloaded kept after them
export LD_PRELOAD="$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)${LD_PRELOAD:+:$LD_PRELOAD}"
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
args=("$@")
[ ${#args[@]} -gt 0 ] || args=(tests/test_cpu_oracle.py tests/test_cpu_plan.py tests/test_cpu_golden.py tests/test_cpu_ifft_model.py)
exec python -m pytest -q -p no:cacheprovider -m "not gpu" "${args[@]}"
