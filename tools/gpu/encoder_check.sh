set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_encoder.py > gpurun_out/encoder_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/encoder_tests.log; exit 1; }
tail -2 gpurun_out/encoder_tests.log
timeout -k 10 400 python -u tools/bench_encoder.py > gpurun_out/bench_encoder.json 2> gpurun_out/bench_encoder.err || { echo BENCH_FAILED; tail -30 gpurun_out/bench_encoder.err; exit 1; }
cat gpurun_out/bench_encoder.json
