set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/profile_pmc.sh gpurun_out/final_c2 || { echo C2_PROFILE_FAILED; exit 1; }
python tools/pmc_summary.py gpurun_out/final_c2 --workload hotpot90k --batch 1024 --out gpurun_out/final_c2/pmc_traffic.json || exit 1
bash tools/profile_pmc.sh gpurun_out/final_c3 --workload synth5m --steps 5 --warmup 2 --no-cpu-baseline --inflight 1 || { echo C3_PROFILE_FAILED; exit 1; }
python tools/pmc_summary.py gpurun_out/final_c3 --workload synth5m --batch 1024 --out gpurun_out/final_c3/pmc_traffic.json || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/final_bench_n1.json 2> gpurun_out/final_bench_n1.err || { echo BENCH_FAIL; tail -20 gpurun_out/final_bench_n1.err; exit 1; }
timeout -k 10 400 python -u bench.py --workload synth5m --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/final_bench_c3.json 2> gpurun_out/final_bench_c3.err || { echo BENCH_C3_FAIL; tail -20 gpurun_out/final_bench_c3.err; exit 1; }
cat gpurun_out/final_c2/pmc_traffic.json | cut -c1-800
python -c "import json; d=json.load(open('gpurun_out/final_bench_n1.json')); print(d['value'], d['roofline'], d['config']['serial_ms_per_step'])"
python -c "import json; d=json.load(open('gpurun_out/final_bench_c3.json')); print(d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
