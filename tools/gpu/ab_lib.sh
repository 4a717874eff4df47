#!/bin/bash
# usage: ab_lib.sh OUT ROUNDS WORKLOAD LIB_A LIB_B
set -o pipefail
O=$1; R=$2; W=$3; A=$4; B=$5
mkdir -p $O
for r in $(seq 1 $R); do
  for v in A B; do
    lib=$A; [ $v == B ] && lib=$B
    AHR_LIB_PATH=$lib timeout -k 10 200 python -u tools/dense_ablation.py --workload $W --batches 1024 --variants prod:-1:0 --rounds 2 > $O/${W}_${v}_r$r.json 2> $O/${W}_${v}_r$r.err || { echo FAIL $v; tail -5 $O/${W}_${v}_r$r.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['prod']['tile_topk'], sum(d['prod'].values()))" $O/${W}_${v}_r$r.json $W $v
  done
done
