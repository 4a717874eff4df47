set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04k; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_qres_gpu.py -x -q --timeout 240 --timeout-method thread > $O/qres_tests.log 2>&1 || { echo QRES_TESTS_FAILED; tail -30 $O/qres_tests.log; exit 1; }
tail -2 $O/qres_tests.log
run() { n=$1; w=$2; shift 2
  env "$@" timeout -k 10 240 python -u tools/qres_trace.py --workload $w --reps 1 --json $O/$n.json > $O/$n.log 2>&1 || { echo FAIL; tail -20 $O/$n.log; exit 1; }
  echo "== $n"; tail -1 $O/$n.log; }
run c2_default hotpot90k AHR_X=0
run d384_default hotpot90k_d384 AHR_X=0
bash tools/gpu/ab_bench.sh $O/ab 2 "--debug-flags 0" "AHR_LIB_PATH=ah-rag_amd/ah_rag/_lib/r03/libahr_hip.so@--debug-flags 0" "--debug-flags 67108864" -- --steps 200 --warmup 20
