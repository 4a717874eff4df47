#!/bin/bash
# Workgroup cap of the 128 x 128 plans (AHR_TILE_SLOTS) at B = 64 / 128 / 256, alternating on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/slots}; mkdir -p $O
for r in 1 2; do
  for v in 512 256 128 64; do
    for b in 64 128 256; do
      f=$O/b${b}_s${v}_r$r
      timeout -k 10 200 env AHR_TILE_SLOTS=$v python -u bench.py --batch $b --steps 1000 --no-sublines --no-f32-line --no-batch-sweep --no-cpu-baseline > $f.json 2> $f.err || { echo FAIL $v $b; tail -5 $f.err; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['config']['serial_ms_per_step'], d['config']['launch'].get('n_splits'), d['stages_ms_per_step'], d['recall_at_10'])" $f.json "slots=$v B=$b r$r"
    done
  done
done
