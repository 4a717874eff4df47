# Register-resident kernel at C2: parity tests, production A/B against the tile kernel (interleaved,
# one process), then the cost split (ablation build: wrong-result switches).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_qres_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/qres_tests.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/qres_tests.log; exit 1; }
tail -2 gpurun_out/qres_tests.log
timeout -k 10 400 python -u tools/dense_ablation.py --batches 1024 --rounds 3 --variants prod:-1:0,tl:-1:32 \
  > gpurun_out/qres_ab.log 2>&1 || { echo AB_FAILED; tail -30 gpurun_out/qres_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/qres_ab.log | tail -3
AHR_LIB_PATH=ah-rag_amd/ah_rag/_lib/ablation/libahr_hip.so timeout -k 10 400 python -u tools/dense_ablation.py --batches 1024 --rounds 3 \
  --variants prod:-1:0,gemm:-1:2,noload:-1:514,nowait:-1:1026,nobar:-1:16778242,noread:-1:33554434,bare:-1:50333186 \
  > gpurun_out/qres_ablation.log 2>&1 || { echo ABL_FAILED; tail -30 gpurun_out/qres_ablation.log; exit 1; }
grep -v amdgpu.ids gpurun_out/qres_ablation.log | tail -3
