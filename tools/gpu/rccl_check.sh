set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_distributed_gpu.py > gpurun_out/rccl_tests.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/rccl_tests.log; exit 1; }
tail -3 gpurun_out/rccl_tests.log
timeout -k 10 400 python -u bench.py --gpus 2 --backend gloo --steps 10 --warmup 3 > gpurun_out/bench_n2_gloo.json 2> gpurun_out/bench_n2_gloo.err || { echo N2_FAILED; tail -30 gpurun_out/bench_n2_gloo.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_n2_gloo.json')); print(d['value'], d['ms_per_step'], d['config']['serial_ms_per_step'], d['config']['inflight'], d['recall_at_10'], d['config']['n1_same_workload_qps'])"
