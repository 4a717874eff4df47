set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for rows in 0 2500000 1250000 625000; do
  timeout -k 10 300 python -u tools/dense_ablation.py --workload synth5m --dtype f16 --rows $rows --batches 1024 --rounds 2 --steps 5 --variants s16k:16384:0,s32k:32768:0,s64k:65536:0 > gpurun_out/sweep_$rows.log 2>&1 || { echo FAIL $rows; tail -5 gpurun_out/sweep_$rows.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/sweep_$rows.log
done
