#!/bin/bash
# B = 64 on the C2 corpus: the threshold pre-pass sample size (0 = no pre-pass) and the forced
# register-resident plan, each a bench line (two batches in flight where the plan allows)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/b64}; mkdir -p $O
for v in "-1 0" "0 0" "2048 0" "4096 0" "-1 8388608"; do
  set -- $v
  timeout -k 10 200 python -u bench.py --batch 64 --steps 1000 --no-sublines --no-f32-line --no-batch-sweep --no-cpu-baseline --sample-rows $1 --debug-flags $2 > $O/s$1_f$2.json 2> $O/s$1_f$2.err || { echo FAIL $v; tail -5 $O/s$1_f$2.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['config']['serial_ms_per_step'], d['config']['launch']['kernel'], d['stages_ms_per_step'], d['recall_at_10'])" $O/s$1_f$2.json "$v"
done
