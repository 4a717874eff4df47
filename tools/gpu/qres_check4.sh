# 16x16x32 forms (8 waves x 32 queries, 4 waves x 64 queries): qres parity, then the cost split.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_qres_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/qres_tests6.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/qres_tests6.log; exit 1; }
tail -1 gpurun_out/qres_tests6.log
AHR_LIB_PATH=ah-rag_amd/ah_rag/_lib/ablation/libahr_hip.so timeout -k 10 400 python -u tools/dense_ablation.py --batches 1024 --rounds 3 \
  --variants p4w:-1:536870912,max4w:-1:536871168,g4w:-1:536870914,nr4w:-1:570425346,p16:-1:268435456,p32:-1:0,g32:-1:2,tl:-1:32 \
  > gpurun_out/qres_ablation18.log 2>&1 || { echo ABL_FAILED; tail -30 gpurun_out/qres_ablation18.log; exit 1; }
grep -v amdgpu.ids gpurun_out/qres_ablation18.log | tail -1
