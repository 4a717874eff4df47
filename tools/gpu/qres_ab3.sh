# Register-resident kernel at C2: threshold-seed sample sizes (production build, tile kernel time =
# survivor cost) and compile-time cost-split variants (ablation build), stagger on / off.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/dense_ablation.py --batches 1024 --rounds 3 \
  --variants p8:8192:0,p16:16384:0,p32:32768:0,l8:8192:67108864,l16:16384:67108864,l32:32768:67108864,tl8:8192:32,tl32:32768:32 \
  > gpurun_out/qres_ab3.log 2>&1 || { echo AB_FAILED; tail -30 gpurun_out/qres_ab3.log; exit 1; }
grep -v amdgpu.ids gpurun_out/qres_ab3.log | tail -1
AHR_LIB_PATH=ah-rag_amd/ah_rag/_lib/ablation/libahr_hip.so timeout -k 10 400 python -u tools/dense_ablation.py --batches 1024 --rounds 3 \
  --variants prod:-1:0,ls:-1:67108864,gemm:-1:2,gemm_ls:-1:67108866,nwb:-1:16778242,nwb_ls:-1:83887106,noread:-1:33554434,noread_ls:-1:100663298,bare:-1:50333186,bare_ls:-1:117442050 \
  > gpurun_out/qres_ablation3.log 2>&1 || { echo ABL_FAILED; tail -30 gpurun_out/qres_ablation3.log; exit 1; }
grep -v amdgpu.ids gpurun_out/qres_ablation3.log | tail -1
