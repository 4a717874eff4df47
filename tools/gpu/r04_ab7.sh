set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04i; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_qres_gpu.py tests/test_dense_gpu.py -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/gpu/ab_bench.sh $O/ab 2 "--debug-flags 0" "--debug-flags 0 --inflight 1" "--debug-flags 67108864" -- --steps 300 --warmup 30
