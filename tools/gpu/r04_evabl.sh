set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04g; mkdir -p $O
A=ah-rag_amd/ah_rag/_lib/ablation/libahr_hip.so
E="AHR_QRES_PUB=ffffffff AHR_QRES_EV=fffffffc"
bash tools/gpu/ab_bench.sh $O/ab 2 "AHR_LIB_PATH=$A@--debug-flags 134217728" "AHR_LIB_PATH=$A $E@--debug-flags 3221225472" "AHR_LIB_PATH=$A $E@--debug-flags 2147483648" "AHR_LIB_PATH=$A $E@--debug-flags 1073741824" "AHR_LIB_PATH=$A $E@--debug-flags 0" -- --steps 200 --warmup 20
