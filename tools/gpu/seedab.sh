#!/bin/bash
# same box: the register-resident kernel self-seeded (default) vs seeded by the sampled pre-pass
# (flag 1 << 26), stage times event-timed, alternating (tools/dense_ablation.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/seedab}; mkdir -p $O
for W in hotpot90k hotpot90k_d384; do
  timeout -k 10 300 python -u tools/dense_ablation.py --workload $W --batches 1024 --variants self:-1:0,prepass:-1:67108864,prepass16k:16384:67108864 --rounds 4 --steps 40 > $O/$W.json 2> $O/$W.err || { echo FAIL; tail -5 $O/$W.err; exit 1; }
  cat $O/$W.json
done
