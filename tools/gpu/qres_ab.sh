#!/bin/bash
# qres A/B of two library builds: the register-resident kernel's GPU tests on the in-tree build,
# then the tile stage alternately at d = 384 and C2 (tools/gpu/ab_libs.sh).
# usage: bash tools/gpu/qres_ab.sh OUT ROUNDS LIB_A LIB_B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$1; R=$2; A=$3; B=$4
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_qres_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu/ab_libs.sh $O/ab $R hotpot90k_d384 $A $B || exit 1
bash tools/gpu/ab_libs.sh $O/ab 2 hotpot90k $A $B || exit 1
