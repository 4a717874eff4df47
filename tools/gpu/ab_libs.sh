#!/bin/bash
# Same-box A/B of several library builds on one workload's default plan, alternating builds each
# round (tile-kernel stage event-timed by tools/dense_ablation.py).
# usage: ab_libs.sh OUT ROUNDS WORKLOAD LIB...   (labels: the libraries' directory names)
set -o pipefail
O=$1; R=$2; W=$3; shift 3
mkdir -p $O
for r in $(seq 1 $R); do
  for lib in "$@"; do
    v=$(basename $(dirname $lib))
    AHR_LIB_PATH=$lib timeout -k 10 200 python -u tools/dense_ablation.py --workload $W --batches 1024 --variants prod:-1:0 --rounds 2 > $O/${W}_${v}_r$r.json 2> $O/${W}_${v}_r$r.err || { echo FAIL $v; tail -5 $O/${W}_${v}_r$r.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['prod']['tile_topk'], round(sum(d['prod'].values()), 4))" $O/${W}_${v}_r$r.json $W $v
  done
done
