#!/bin/bash
# The round-end set on one box: every -m gpu test (parity margins kept), smoke, the default bench
# line, the bench + rocprofv3 kernel trace of the same workload, PMC passes for C2 and C3.
# usage: bash tools/gpu/final.sh [OUTDIR]
set -o pipefail
cd $GRAFT_REPO_ROOT
AHR_PARITY_LOG=${1:-gpurun_out/final}/check/parity_margins.jsonl bash tools/gpu/check.sh ${1:-gpurun_out/final}/check || exit 1
bash tools/gpu/trace.sh ${1:-gpurun_out/final}/c2_trace || exit 1
bash tools/gpu/profile.sh ${1:-gpurun_out/final}/final_c2 hotpot90k || exit 1
bash tools/gpu/profile.sh ${1:-gpurun_out/final}/final_c3 synth5m || exit 1
