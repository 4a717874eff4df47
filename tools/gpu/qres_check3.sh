# 16x16x32 form with staged screening: qres parity, then the cost split against the 32x32 form.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_qres_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/qres_tests5.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/qres_tests5.log; exit 1; }
tail -1 gpurun_out/qres_tests5.log
AHR_LIB_PATH=ah-rag_amd/ah_rag/_lib/ablation/libahr_hip.so timeout -k 10 400 python -u tools/dense_ablation.py --batches 1024 --rounds 3 \
  --variants p16:-1:268435456,max16:-1:268435712,st16:-1:402653184,p32:-1:0,tl:-1:32 \
  > gpurun_out/qres_ablation17.log 2>&1 || { echo ABL_FAILED; tail -30 gpurun_out/qres_ablation17.log; exit 1; }
grep -v amdgpu.ids gpurun_out/qres_ablation17.log | tail -1
