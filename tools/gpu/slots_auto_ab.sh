#!/bin/bash
# Automatic tile-plan workgroup cap (256 with several reserved workspaces) vs fixed 512, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/slots_auto}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_dense_gpu.py tests/test_configs_gpu.py tests/test_probe_seed_gpu.py tests/test_distributed_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAIL; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for e in "AHR_TILE_SLOTS=512" "AHR_TILE_SLOTS=0"; do
    for b in 64 128 256; do
      f=$O/b${b}_${e#AHR_TILE_SLOTS=}_r$r
      timeout -k 10 200 env $e python -u bench.py --batch $b --steps 1000 --no-sublines --no-f32-line --no-batch-sweep --no-cpu-baseline > $f.json 2> $f.err || { echo FAIL $e $b; tail -5 $f.err; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['config']['serial_ms_per_step'], d['config']['launch'].get('n_splits'), d['recall_at_10'])" $f.json "$e B=$b r$r"
    done
  done
done
