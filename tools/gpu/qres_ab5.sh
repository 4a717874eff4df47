# 16x16x32 register-resident kernel: parity tests, A/B against the 32x32x16 form and the tile
# kernels (production build, interleaved), cost split (ablation build).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_qres_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/qres_tests.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/qres_tests.log; exit 1; }
tail -1 gpurun_out/qres_tests.log
timeout -k 10 400 python -u tools/dense_ablation.py --batches 1024 --rounds 4 \
  --variants q16:-1:0,q32:-1:268435456,tl:-1:32,t256:-1:32768 \
  > gpurun_out/qres_ab6.log 2>&1 || { echo AB_FAILED; tail -30 gpurun_out/qres_ab6.log; exit 1; }
grep -v amdgpu.ids gpurun_out/qres_ab6.log | tail -1
AHR_LIB_PATH=ah-rag_amd/ah_rag/_lib/ablation/libahr_hip.so timeout -k 10 400 python -u tools/dense_ablation.py --batches 1024 --rounds 3 \
  --variants prod:-1:0,gemm:-1:2,nwb:-1:16778242,noread:-1:33554434,bare:-1:50333186 \
  > gpurun_out/qres_ablation6.log 2>&1 || { echo ABL_FAILED; tail -30 gpurun_out/qres_ablation6.log; exit 1; }
grep -v amdgpu.ids gpurun_out/qres_ablation6.log | tail -1
