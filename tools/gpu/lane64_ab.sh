#!/bin/bash
# 256 x 64 lane plan (AHR_LANE64=1) vs the 128 x 128 tile plan at 17 <= B <= 64: parity under the
# plan, then bench lines alternating on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/lane64}; mkdir -p $O
AHR_LANE64=1 timeout -k 10 600 python -u -m pytest tests/test_dense_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -rs > $O/tests.log 2>&1 || { echo TESTS FAIL; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for r in 1 2; do
  for e in 0 1; do
    for b in 64 32; do
      f=$O/b${b}_l${e}_r$r
      timeout -k 10 200 env AHR_LANE64=$e python -u bench.py --batch $b --steps 1000 --no-sublines --no-f32-line --no-batch-sweep --no-cpu-baseline > $f.json 2> $f.err || { echo FAIL $e $b; tail -5 $f.err; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['config']['serial_ms_per_step'], d['config']['launch'], d['stages_ms_per_step'].get('tile_topk'), d['recall_at_10'])" $f.json "lane64=$e B=$b r$r"
    done
  done
done
