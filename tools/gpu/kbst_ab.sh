set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_dense_gpu.py -k "loader or kb256" > gpurun_out/kbst_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/kbst_tests.log; exit 1; }
tail -2 gpurun_out/kbst_tests.log
timeout -k 10 500 python -u tools/dense_ablation.py --workload synth5m --dtype f16 --batches 1024 --rounds 3 --steps 5 --variants prod:-1:0,ld:-1:2097152,gemm:-1:2,gemm_ld:-1:2097154,noload:-1:514 > gpurun_out/kbst_ab.log 2>&1 || { echo ABL_FAILED; tail -30 gpurun_out/kbst_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/kbst_ab.log
