#!/bin/bash
# Automatic tile cap at fp32 B = 64 / 256 (two in flight) vs fixed 512, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/slots_f32b}; mkdir -p $O
for r in 1 2; do
  for v in 512 0; do
    for b in 64 256; do
      f=$O/f32_b${b}_s${v}_r$r
      timeout -k 10 200 env AHR_TILE_SLOTS=$v python -u bench.py --batch $b --dtype f32 --steps 500 --no-sublines --no-f32-line --no-batch-sweep --no-cpu-baseline > $f.json 2> $f.err || { echo FAIL $v $b; tail -5 $f.err; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['config']['serial_ms_per_step'], d['config']['launch'].get('n_splits'))" $f.json "slots=$v f32 B=$b r$r"
    done
  done
done
