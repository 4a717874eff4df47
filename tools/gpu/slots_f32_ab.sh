#!/bin/bash
# The default bench's C2, exact-fp32 and batch-sweep lines under the automatic tile cap vs fixed 512
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/slots_f32}; mkdir -p $O
for r in 1 2; do
  for e in "AHR_TILE_SLOTS=512" "AHR_TILE_SLOTS=0"; do
    f=$O/default_${e#AHR_TILE_SLOTS=}_r$r
    timeout -k 10 300 env $e python -u bench.py --no-sublines --no-cpu-baseline > $f.json 2> $f.err || { echo FAIL $e; tail -5 $f.err; exit 1; }
    python -c "
import json,sys; d=json.load(open(sys.argv[1])); f=d['exact_fp32']
print(sys.argv[2], 'C2', d['value'], 'f32', f.get('value'), f.get('ms_per_step'), (f.get('config') or {}).get('launch'), [(b['batch'], b['ms_per_step']) for b in d['batch_sweep']])" $f.json "$e r$r"
  done
done
