#!/bin/bash
# Same-box A/B/... of library builds on B = 1024 steps (alternating builds, dense_ablation prod stage times).
# usage: ab_libsn.sh OUT ROUNDS "WORKLOADS" LIB_1 LIB_2 ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$1; R=$2; WS=$3; shift 3
mkdir -p $O
for r in $(seq 1 $R); do
  for W in $WS; do
    i=0
    for lib in "$@"; do
      i=$((i+1))
      st=20; [ $W == synth5m ] && st=8
      AHR_LIB_PATH=$lib timeout -k 10 200 python -u tools/dense_ablation.py --workload $W --batches 1024 --variants prod:-1:0 --rounds 2 --steps $st > $O/${W}_v${i}_r$r.json 2> $O/${W}_v${i}_r$r.err || { echo FAIL $lib; tail -5 $O/${W}_v${i}_r$r.err; exit 1; }
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['prod']['tile_topk'], round(sum(d['prod'].values()),4))" $O/${W}_v${i}_r$r.json $W v$i
    done
  done
done
