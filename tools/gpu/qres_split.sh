#!/bin/bash
# Cost split and per-workgroup timeline of the register-resident kernel on one workload, from the
# ablation build (copy ah-rag_amd/ah_rag/_lib/ablation to _lib/abl first: _lib/ablation is not uploaded).
# usage: bash tools/gpu/qres_split.sh OUT WORKLOAD
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$1; W=$2
mkdir -p $O
L=$PWD/ah-rag_amd/ah_rag/_lib/abl/libahr_hip.so
V="prod:-1:0,noscreen:-1:2,nobarrier:-1:16777216,nowait_nobar:-1:17826816,gemm_noloads:-1:514,gemm_core:-1:50333186"
AHR_LIB_PATH=$L timeout -k 10 300 python -u tools/dense_ablation.py --workload $W --batches 1024 --rounds 3 --variants $V > $O/split_$W.json 2> $O/split_$W.err || { echo SPLIT_FAIL; tail -5 $O/split_$W.err; exit 1; }
tail -1 $O/split_$W.json | cut -c1-900
AHR_LIB_PATH=$L timeout -k 10 300 python -u tools/qres_trace.py --workload $W --json $O/timeline_$W.json > $O/timeline_$W.txt 2> $O/timeline_$W.err || { echo TRACE_FAIL; tail -5 $O/timeline_$W.err; exit 1; }
head -30 $O/timeline_$W.txt
