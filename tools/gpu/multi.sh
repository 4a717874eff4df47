#!/bin/bash
# Multi-rank checks on one box: the RCCL tests, then 2-rank gloo rehearsals of the row-sharded
# bench and of the C5 replicas mode (two ranks share the card: correctness, not scaling data).
# usage: bash tools/gpu/multi.sh [OUTDIR]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/multi}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_distributed_gpu.py > $O/rccl_tests.log 2>&1 || { echo TESTS_FAILED; tail -60 $O/rccl_tests.log; exit 1; }
tail -3 $O/rccl_tests.log
timeout -k 10 400 python -u bench.py --gpus 2 --backend gloo --steps 10 --warmup 3 > $O/bench_n2_gloo.json 2> $O/bench_n2_gloo.err || { echo N2_FAILED; tail -30 $O/bench_n2_gloo.err; exit 1; }
cut -c1-600 $O/bench_n2_gloo.json
timeout -k 10 300 python -u bench.py --gpus 2 --backend gloo --workload env > $O/bench_env_n2.json 2> $O/bench_env_n2.err || { echo ENV_FAILED; tail -30 $O/bench_env_n2.err; exit 1; }
cut -c1-600 $O/bench_env_n2.json
