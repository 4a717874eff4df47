# Round-3 profiles: C2 (qres256) and C3 (kb256) kernel traces, HBM traffic and SQ (MFMA busy) passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/profile_pmc.sh gpurun_out/r03_c2 || { echo C2_PROFILE_FAILED; exit 1; }
python tools/pmc_summary.py gpurun_out/r03_c2 --workload hotpot90k --batch 1024 --out gpurun_out/r03_c2/pmc_traffic.json || exit 1
bash tools/profile_pmc.sh gpurun_out/r03_c3 --workload synth5m --steps 5 --warmup 2 --no-cpu-baseline --inflight 1 --no-batch-sweep || { echo C3_PROFILE_FAILED; exit 1; }
python tools/pmc_summary.py gpurun_out/r03_c3 --workload synth5m --batch 1024 --out gpurun_out/r03_c3/pmc_traffic.json || exit 1
