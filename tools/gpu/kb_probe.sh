set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/dense_ablation.py --workload synth5m --dtype f16 --batches 1024 --rounds 3 --steps 5 --variants prod:-1:0,gemm:-1:2,max:-1:256,noload:-1:514,nowait:-1:1026 > gpurun_out/kb_probe.log 2>&1 || { echo ABL_FAILED; tail -30 gpurun_out/kb_probe.log; exit 1; }
grep -v amdgpu.ids gpurun_out/kb_probe.log
