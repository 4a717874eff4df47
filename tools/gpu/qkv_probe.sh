set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/dense_ablation.py --batches 1024,2048 --rounds 4 --variants prod:-1:0,qkv:-1:4096,qkv_gemm:-1:4098,qkv_max:-1:4352,qkv_noload:-1:4610,tl_gemm:-1:34,tl_noload:-1:546,t256_gemm:-1:32770 > gpurun_out/qkv_probe.log 2>&1 || { echo ABL_FAILED; tail -30 gpurun_out/qkv_probe.log; exit 1; }
grep -v amdgpu.ids gpurun_out/qkv_probe.log
