set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_distributed_gpu.py > gpurun_out/rccl_tests.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/rccl_tests.log; exit 1; }
tail -3 gpurun_out/rccl_tests.log
