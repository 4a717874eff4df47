#!/bin/bash
# Small-batch kernel split count (AHR_SMALL_SPLITS) at B = 1 / 4 / 16, bf16 and fp32, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/small_splits}; mkdir -p $O
for r in 1 2; do
  for v in 256 128 512; do
    for c in "bf16 1" "bf16 16" "f32 1" "f32 4"; do
      set -- $c
      f=$O/${1}_b$2_s${v}_r$r
      timeout -k 10 200 env AHR_SMALL_SPLITS=$v python -u bench.py --batch $2 --dtype $1 --steps 2000 --no-sublines --no-f32-line --no-batch-sweep --no-cpu-baseline > $f.json 2> $f.err || { echo FAIL $v $c; tail -5 $f.err; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['config']['serial_ms_per_step'], d['config']['launch'].get('n_splits'))" $f.json "splits=$v $c r$r"
    done
  done
done
