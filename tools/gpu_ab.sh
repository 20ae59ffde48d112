#!/bin/bash
# A/B of a kernel variant switch: GPU parity suite (default variant), then a kernel trace of the
# bench with the default and with the env switch $2 (e.g. DVBT2LL_BCH_V1=1) set.
# Usage: tools/gpu_ab.sh TAG VAR=VALUE [extra bench args]
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
T=$1; V=$2; shift 2
NOBENCH=1 bash tools/gpu_check.sh "$T" || exit $?
bash tools/gpu_trace.sh "$T/a" "$@" || exit $?
export "$V"
bash tools/gpu_trace.sh "$T/b" "$@"
