#!/bin/bash
# Round-5 fourth pass: qres GPU tests on the current library, then A/B of the committed build,
# the branchless quad appends (d = 384) and those plus the coarse seeding grid.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/r5d}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_qres_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 || { echo TESTS_FAILED; tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
L=$PWD/ah-rag_amd/ah_rag/_lib
for W in hotpot90k_d384 hotpot90k; do bash tools/gpu/ab_libs.sh $O/ab_$W 3 $W $L/base2/libahr_hip.so $L/blonly/libahr_hip.so $L/libahr_hip.so || exit 1; done
