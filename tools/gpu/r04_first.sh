set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04a
timeout -k 10 600 python -u -m pytest tests/test_qres_gpu.py -x -v --timeout 240 --timeout-method thread > gpurun_out/r04a/qres_tests.log 2>&1; rc=$?
tail -5 gpurun_out/r04a/qres_tests.log
[ $rc -eq 0 ] || { echo QRES_TESTS_FAILED; grep -E 'FAILED|Error|assert' gpurun_out/r04a/qres_tests.log | head -20; exit 1; }
bash tools/gpu/ab_bench.sh gpurun_out/r04a/ab 2 "--debug-flags 0" "--debug-flags 67108864" -- --steps 200 --warmup 20
