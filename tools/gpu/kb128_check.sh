set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_dense_gpu.py -k "kb128 or kb256 or tl16" > gpurun_out/kb128_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/kb128_tests.log; exit 1; }
tail -2 gpurun_out/kb128_tests.log
timeout -k 10 300 python -u tools/dense_ablation.py --batches 1024,4096 --rounds 3 --variants prod:-1:0,tl_gemm:-1:34,tl_max:-1:288,tl16:-1:1048576,tl16_gemm:-1:1048578,tl16_max:-1:1048832,kb128:-1:524288 > gpurun_out/kb128_ablation.log 2>&1
grep -v amdgpu.ids gpurun_out/kb128_ablation.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_new.json 2> gpurun_out/bench_new.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench_new.err; exit 1; }
python -c "import json; d=json.load(open(\"gpurun_out/bench_new.json\")); print(d[\"value\"], d[\"exact_fp32\"], d[\"cpu_baseline\"][\"value\"], d[\"cpu_baseline\"][\"cores\"], d[\"cpu_baseline\"][\"b1024_queries_per_s_by_blas_threads\"])"
