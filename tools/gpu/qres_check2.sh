# Register-resident kernel: parity (qres + dense + C2 configs), then the two forms' cost split.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_qres_gpu.py tests/test_dense_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread -k "not c3 and not c4" --deselect tests/test_dense_gpu.py::test_default_plans > gpurun_out/qres_tests.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/qres_tests.log; exit 1; }
tail -1 gpurun_out/qres_tests.log
AHR_LIB_PATH=ah-rag_amd/ah_rag/_lib/ablation/libahr_hip.so timeout -k 10 400 python -u tools/dense_ablation.py --batches 1024 --rounds 3 \
  --variants p16:-1:268435456,g16:-1:268435458,nr16:-1:301989890,p32:-1:0,g32:-1:2,nr32:-1:33554434,bare32:-1:50333186,tl:-1:32 \
  > gpurun_out/qres_ablation11.log 2>&1 || { echo ABL_FAILED; tail -30 gpurun_out/qres_ablation9.log; exit 1; }
grep -v amdgpu.ids gpurun_out/qres_ablation11.log | tail -1
