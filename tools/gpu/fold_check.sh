set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_small_fold_gpu.py tests/test_dense_gpu.py -k "fold or small" > gpurun_out/fold_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/fold_tests.log; exit 1; }
tail -1 gpurun_out/fold_tests.log
timeout -k 10 300 python -u tools/fold_latency.py > gpurun_out/fold_latency.log 2>&1 || { tail -20 gpurun_out/fold_latency.log; exit 1; }
tail -1 gpurun_out/fold_latency.log
