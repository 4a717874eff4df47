set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_dense_gpu.py -k "screening_forms or ties or prepass" > gpurun_out/screen_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/screen_tests.log; exit 1; }
tail -2 gpurun_out/screen_tests.log
timeout -k 10 300 python -u tools/dense_ablation.py --batches 1024 --rounds 5 --variants prod:-1:0,v4:-1:67108864,v2q:-1:10485760,tl_max:-1:288,tl_gemm:-1:34 > gpurun_out/screen_ablation.log 2>&1 || { echo ABL_FAILED; tail -30 gpurun_out/screen_ablation.log; exit 1; }
grep -v amdgpu.ids gpurun_out/screen_ablation.log
