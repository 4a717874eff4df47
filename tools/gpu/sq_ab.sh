#!/bin/bash
# SQ counter passes of the C2 register-resident launch: production vs GEMM-only (ablation flag 2)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/sq_ab}; mkdir -p $O
export AHR_LIB_PATH=ah-rag_amd/ah_rag/_lib/ablation/libahr_hip.so
B="--steps 10 --warmup 3 --clock-ramp 20 --no-cpu-baseline --no-sublines --no-batch-sweep --no-f32-line --inflight 1"
bash tools/profile_sq.sh $O/prod $B || exit 1
bash tools/profile_sq.sh $O/gemm $B --debug-flags 2 || exit 1
for v in prod gemm; do echo $v; python tools/sq_summary.py $O/$v --kernel topk_qres; done
