#!/bin/bash
# Traffic attribution of the register-resident kernel: the same launches seeded by the sampled
# pre-pass (flag 1 << 26: no publications, no granule / seed reads) beside the self-seeded default,
# FETCH_SIZE / WRITE_SIZE passes; then a seeding-schedule re-check at C2 on the 16x16x32 build.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/attrib}; mkdir -p $O
for W in hotpot90k hotpot90k_d384; do
  bash tools/gpu/profile.sh $O/${W}_prepass $W --debug-flags 67108864 > $O/${W}_prepass.txt 2>&1 || { echo PROF_FAIL; tail -5 $O/${W}_prepass.txt; exit 1; }
done
bash tools/gpu/ab_env.sh $O/sched 2 hotpot90k "-" "AHR_QRES_PUB=55555555 AHR_QRES_EV=aaaaaaaa" "AHR_QRES_PUB=44444455 AHR_QRES_EV=88888aa8" "AHR_QRES_PUB=40404055 AHR_QRES_EV=808080a8" || exit 1
