# 32x32x16 qres with one barrier per block (flag 1 << 31) instead of one per stage: parity, then time.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_qres_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/qres_blk_tests.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/qres_blk_tests.log; exit 1; }
tail -1 gpurun_out/qres_blk_tests.log
AHR_LIB_PATH=ah-rag_amd/ah_rag/_lib/ablation/libahr_hip.so timeout -k 10 400 python -u tools/dense_ablation.py --batches 1024 --rounds 3 \
  --variants p32:-1:0,p2p:-1:2147483648,g32:-1:2,g2p:-1:2147483650,p32b:-1:0,p2pb:-1:2147483648 \
  > gpurun_out/qres_blk.log 2>&1 || { echo ABL_FAILED; tail -30 gpurun_out/qres_blk.log; exit 1; }
grep -v amdgpu.ids gpurun_out/qres_blk.log | tail -1
