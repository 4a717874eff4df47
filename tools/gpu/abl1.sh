set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/abl1; mkdir -p $O
for W in synth5m hotpot90k hotpot90k_d384; do
  AHR_LIB_PATH=ah-rag_amd/ah_rag/_lib/ablation/libahr_hip.so timeout -k 10 300 python -u tools/dense_ablation.py --workload $W --batches 1024 --variants prod:-1:0,gemm:-1:2 --rounds 2 --steps 20 > $O/$W.json 2> $O/$W.err || { echo FAIL $W; tail -5 $O/$W.err; exit 1; }
  tail -1 $O/$W.json
done
