#!/bin/bash
# Same-box A/B of two library builds on the C2, C3 and d = 384 B = 1024 steps (alternating builds).
# usage: ab_libs3.sh OUT ROUNDS LIB_A LIB_B [WORKLOADS]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$1; R=$2; A=$3; B=$4; WS=${5:-"hotpot90k synth5m hotpot90k_d384"}
mkdir -p $O
for r in $(seq 1 $R); do
  for W in $WS; do
    for v in A B; do
      lib=$A; [ $v == B ] && lib=$B
      st=20; [ $W == synth5m ] && st=8
      AHR_LIB_PATH=$lib timeout -k 10 200 python -u tools/dense_ablation.py --workload $W --batches 1024 --variants prod:-1:0 --rounds 2 --steps $st > $O/${W}_${v}_r$r.json 2> $O/${W}_${v}_r$r.err || { echo FAIL $v; tail -5 $O/${W}_${v}_r$r.err; exit 1; }
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['prod']['tile_topk'], round(sum(d['prod'].values()),4))" $O/${W}_${v}_r$r.json $W $v
    done
  done
done
