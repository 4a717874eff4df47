set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04c
timeout -k 10 300 python -u -m pytest tests/test_qres_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r04c/qres_tests.log 2>&1 || { echo QRES_TESTS_FAILED; tail -30 gpurun_out/r04c/qres_tests.log; exit 1; }
tail -2 gpurun_out/r04c/qres_tests.log
bash tools/gpu/ab_bench.sh gpurun_out/r04c/ab 2 "--debug-flags 0" "--debug-flags 67108864" "--debug-flags 335544320" "AHR_LIB_PATH=ah-rag_amd/ah_rag/_lib/r03/libahr_hip.so@--debug-flags 0" "AHR_QRES_PUB=40404457 AHR_QRES_EV=808088ac@--debug-flags 0" "AHR_QRES_PUB=40004011 AHR_QRES_EV=80008020@--debug-flags 0" "AHR_QRES_PUB=40404115 AHR_QRES_EV=80808228@--debug-flags 0" -- --steps 200 --warmup 20
bash tools/gpu/ab_bench.sh gpurun_out/r04c/c3 1 "--debug-flags 0" "--debug-flags 8388608" -- --workload synth5m --steps 10 --warmup 2
