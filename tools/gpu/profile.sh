#!/bin/bash
# rocprofv3 kernel trace + PMC passes (HBM bytes, MFMA busy) and their summary for one workload.
# usage: [BATCH=B] bash tools/gpu/profile.sh OUTDIR WORKLOAD(hotpot90k|hotpot90k_d384|synth5m) [extra bench args]
# (BATCH: the batch the extra args give bench.py, e.g. BATCH=1 DT=0 ... hotpot90k --dtype f32 --batch 1;
#  DT: the storage type of the measured launches, 0 f32 / 1 f16 / 2 bf16, default the workload's)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$1; W=$2; shift 2
mkdir -p $O
if [ "$W" == "synth5m" ]; then STEPS="--steps 5 --warmup 2"; else STEPS="--steps 10 --warmup 3"; fi
bash tools/profile_pmc.sh $O --workload $W $STEPS --no-cpu-baseline --inflight 1 --no-batch-sweep --no-f32-line --no-sublines "$@" || { echo PROFILE_FAILED; exit 1; }
python tools/pmc_summary.py $O --workload $W --batch ${BATCH:-1024} ${DT:+--dt $DT} --out $O/pmc_traffic.json || exit 1
cut -c1-800 $O/pmc_traffic.json
