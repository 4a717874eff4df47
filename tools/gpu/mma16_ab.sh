#!/bin/bash
# Same-box A/B of the register-resident kernel's GEMM core (GEMM-only switch, flag 2): the shipped
# 32x32x16 chain vs the 16x16x32 diagnostic form (AHR_QRES_MMA16 build), alternating builds.
# usage: mma16_ab.sh OUT ROUNDS
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$1; R=${2:-3}; mkdir -p $O
for r in $(seq 1 $R); do
  for v in ablation ablation16; do
    for W in hotpot90k hotpot90k_d384; do
      AHR_LIB_PATH=ah-rag_amd/ah_rag/_lib/$v/libahr_hip.so timeout -k 10 200 python -u tools/dense_ablation.py --workload $W --batches 1024 --variants gemm:-1:2 --rounds 2 --steps 40 > $O/${W}_${v}_r$r.json 2> $O/${W}_${v}_r$r.err || { echo FAIL $v; tail -5 $O/${W}_${v}_r$r.err; exit 1; }
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['gemm']['tile_topk'])" $O/${W}_${v}_r$r.json $W $v
    done
  done
done
