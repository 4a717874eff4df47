# First GPU run of the register-resident kernel: its parity tests, then C2 A/B against the tile
# kernel (same binary, debug flag 32 = tilelane) with stage timings.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_qres_gpu.py -x -v --timeout 240 --timeout-method thread > gpurun_out/qres_tests.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/qres_tests.log; exit 1; }
tail -3 gpurun_out/qres_tests.log
for f in 0 32 0 32; do
  timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-f32-line --no-batch-sweep --debug-flags $f > gpurun_out/ab_$f.json 2> gpurun_out/ab_$f.err || { echo BENCH_FAIL $f; tail -20 gpurun_out/ab_$f.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab_$f.json')); print($f, d['value'], d['roofline']['kernel'][:40], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['config']['serial_ms_per_step'], d['stages_ms_per_step'], d['recall_at_10'])"
done
