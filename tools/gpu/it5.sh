#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/it5}; mkdir -p $O
timeout -k 10 30 ./tools/permlane_probe > $O/permlane.txt 2>&1 && cat $O/permlane.txt || { echo PROBE_FAIL; exit 1; }
bash tools/gpu/bench_libs.sh $O/c2 2 "" ah-rag_amd/ah_rag/_lib/libahr_hip.so ah-rag_amd/ah_rag/_lib/variant_mma32/libahr_hip.so || exit 1
BENCH_ARGS="--workload hotpot90k_d384" bash tools/gpu/bench_libs.sh $O/d384 2 none ah-rag_amd/ah_rag/_lib/libahr_hip.so ah-rag_amd/ah_rag/_lib/variant_mma32/libahr_hip.so || exit 1
BENCH_ARGS="--workload synth5m --steps 20 --warmup 3 --clock-ramp 5" bash tools/gpu/bench_libs.sh $O/c3 1 none ah-rag_amd/ah_rag/_lib/libahr_hip.so ah-rag_amd/ah_rag/_lib/variant_mma32/libahr_hip.so || exit 1
