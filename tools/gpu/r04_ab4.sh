set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04d; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_qres_gpu.py -x -q --timeout 240 --timeout-method thread > $O/qres_tests.log 2>&1 || { echo QRES_TESTS_FAILED; tail -30 $O/qres_tests.log; exit 1; }
tail -2 $O/qres_tests.log
bash tools/gpu/ab_bench.sh $O/ab 2 "--debug-flags 0" "AHR_QRES_PUB=55555555 AHR_QRES_EV=aaaaaaa8@--debug-flags 0" "AHR_QRES_PUB=ffffffff AHR_QRES_EV=fffffffc@--debug-flags 0" "AHR_QRES_PUB=40404455 AHR_QRES_EV=808088a8@--debug-flags 0" "--debug-flags 67108864" -- --steps 200 --warmup 20
