#!/bin/bash
# The round-end set on one box: every -m gpu test (parity margins kept), smoke, the default bench
# line, the bench + rocprofv3 kernel trace of the same workload, PMC passes for C2, C3, d = 384 and
# the drop-in default (fp32, B = 1).
# usage: bash tools/gpu/final.sh [OUTDIR]
set -o pipefail
cd $GRAFT_REPO_ROOT
AHR_PARITY_LOG=${1:-gpurun_out/final}/check/parity_margins.jsonl bash tools/gpu/check.sh ${1:-gpurun_out/final}/check || exit 1
bash tools/gpu/trace.sh ${1:-gpurun_out/final}/c2_trace || exit 1
bash tools/gpu/profile.sh ${1:-gpurun_out/final}/final_c2 hotpot90k || exit 1
bash tools/gpu/profile.sh ${1:-gpurun_out/final}/final_c3 synth5m || exit 1
bash tools/gpu/profile.sh ${1:-gpurun_out/final}/final_d384 hotpot90k_d384 || exit 1
BATCH=1 DT=0 bash tools/gpu/profile.sh ${1:-gpurun_out/final}/final_f32b1 hotpot90k --dtype f32 --batch 1 || exit 1
BATCH=1024 DT=0 bash tools/gpu/profile.sh ${1:-gpurun_out/final}/final_f32 hotpot90k --dtype f32 || exit 1
BATCH=64 bash tools/gpu/profile.sh ${1:-gpurun_out/final}/final_b64 hotpot90k --batch 64 || exit 1
BATCH=1 bash tools/gpu/profile.sh ${1:-gpurun_out/final}/final_b1 hotpot90k --batch 1 || exit 1
