#!/bin/bash
# A/B of environment settings (e.g. the self-seeding schedule) on one workload's dense search stages,
# alternating, one box: tools/gpu/ab_env.sh OUT ROUNDS WORKLOAD "ENV_A" "ENV_B" ...  (ENV: "K=V K=V" or "-")
set -o pipefail
O=$1; R=$2; W=$3; shift 3
mkdir -p $O
for r in $(seq 1 $R); do
  i=0
  for e in "$@"; do
    envs=""; [ "$e" != "-" ] && envs=$e
    timeout -k 10 200 env $envs python -u tools/dense_ablation.py --workload $W --batches 1024 --variants prod:-1:0 --rounds 2 > $O/${W}_v${i}_r$r.json 2> $O/${W}_v${i}_r$r.err || { echo FAIL "$e"; tail -5 $O/${W}_v${i}_r$r.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['prod']['tile_topk'], round(sum(d['prod'].values()), 4))" $O/${W}_v${i}_r$r.json "$W v$i [$e]"
    i=$((i + 1))
  done
done
