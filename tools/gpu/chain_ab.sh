#!/bin/bash
# qres batches on two streams: whole batches ordered (AHR_QRES_CHAIN=merge) vs only the kernels
# (=kernel), against one batch in flight; the two-stream parity test first.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/chain_ab}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_dense_gpu.py tests/test_qres_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu/ab_bench.sh $O/c2 ${2:-2} "AHR_QRES_CHAIN=merge@--inflight 1" "AHR_QRES_CHAIN=merge@--inflight 2" "AHR_QRES_CHAIN=kernel@--inflight 2" "AHR_QRES_CHAIN=kernel@--inflight 3"
