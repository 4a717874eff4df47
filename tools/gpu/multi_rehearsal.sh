set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --gpus 2 --backend gloo --steps 10 --warmup 3 > gpurun_out/bench_n2_gloo.json 2> gpurun_out/bench_n2_gloo.err || { echo N2_FAILED; tail -30 gpurun_out/bench_n2_gloo.err; exit 1; }
cat gpurun_out/bench_n2_gloo.json | cut -c1-600
timeout -k 10 300 python -u tools/bench_env.py --gpus 2 --backend gloo > gpurun_out/bench_env_n2.json 2> gpurun_out/bench_env_n2.err || { echo ENV_FAILED; tail -30 gpurun_out/bench_env_n2.err; exit 1; }
cat gpurun_out/bench_env_n2.json | cut -c1-600
