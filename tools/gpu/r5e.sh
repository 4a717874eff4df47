#!/bin/bash
# Round-5 fifth pass: self-seeding schedule sweep at C2 and d = 384 (same box, alternating), and the
# seed-quality sweep with the first-event-only and unseeded forms.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/r5e}
mkdir -p $O
for W in hotpot90k hotpot90k_d384; do
  bash tools/gpu/ab_env.sh $O/sched_$W 2 $W "-" "AHR_QRES_PUB=40004041 AHR_QRES_EV=80008082" "AHR_QRES_PUB=4001 AHR_QRES_EV=8002" "AHR_QRES_PUB=55555555 AHR_QRES_EV=aaaaaaaa" || exit 1
done
timeout -k 10 400 python -u tools/seed_floor.py --rounds 2 > $O/seed_floor.json 2> $O/seed_floor.err || { echo SEED_FLOOR_FAIL; tail -5 $O/seed_floor.err; exit 1; }
cat $O/seed_floor.json
