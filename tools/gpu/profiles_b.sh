#!/bin/bash
# part B (the fp32 lines and B = 64)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${1:-gpurun_out/final}
BATCH=1 DT=0 bash tools/gpu/profile.sh $O/final_f32b1 hotpot90k --dtype f32 --batch 1 || exit 1
BATCH=1024 DT=0 bash tools/gpu/profile.sh $O/final_f32 hotpot90k --dtype f32 || exit 1
BATCH=64 bash tools/gpu/profile.sh $O/final_b64 hotpot90k --batch 64 || exit 1
