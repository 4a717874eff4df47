#!/bin/bash
# the PMC / trace profiles of the final set, part A (C2, C3, d = 384)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${1:-gpurun_out/final}
bash tools/gpu/profile.sh $O/final_c2 hotpot90k || exit 1
bash tools/gpu/profile.sh $O/final_c3 synth5m || exit 1
bash tools/gpu/profile.sh $O/final_d384 hotpot90k_d384 || exit 1
