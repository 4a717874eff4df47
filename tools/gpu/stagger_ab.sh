set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_dense_gpu.py -k "stagger" > gpurun_out/stagger_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/stagger_tests.log; exit 1; }
tail -2 gpurun_out/stagger_tests.log
timeout -k 10 300 python -u tools/dense_ablation.py --batches 1024 --rounds 5 --variants prod:-1:0,hw:-1:4194304,bid:-1:8388608,gemm:-1:2,gemm_hw:-1:4194306,gemm_bid:-1:8388610 > gpurun_out/stagger_c2.log 2>&1 || { echo ABL_FAILED; tail -30 gpurun_out/stagger_c2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/stagger_c2.log
timeout -k 10 400 python -u tools/dense_ablation.py --workload synth5m --dtype f16 --rows 1250000 --batches 1024 --rounds 4 --steps 10 --variants prod:-1:0,kbst:-1:2097152,gemm:-1:2,gemm_st:-1:2097154 > gpurun_out/stagger_kb.log 2>&1 || { echo ABL_FAILED; tail -30 gpurun_out/stagger_kb.log; exit 1; }
grep -v amdgpu.ids gpurun_out/stagger_kb.log
