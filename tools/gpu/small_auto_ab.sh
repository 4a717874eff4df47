#!/bin/bash
# Small-batch split count: automatic (128 with several workspaces at fp32 B = 4 / half B = 16) vs 256
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/small_auto}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_dense_gpu.py tests/test_configs_gpu.py tests/test_dropin_gpu.py tests/test_c5_env_gpu.py -m gpu -x -q --timeout 250 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in 256 0; do
    for c in "f32 2" "f32 4" "bf16 8" "bf16 16"; do
      set -- $c
      f=$O/${1}_b$2_s${v}_r$r
      timeout -k 10 200 env AHR_SMALL_SPLITS=$v python -u bench.py --batch $2 --dtype $1 --steps 2000 --no-sublines --no-f32-line --no-batch-sweep --no-cpu-baseline > $f.json 2> $f.err || { echo FAIL $v $c; tail -5 $f.err; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['config']['serial_ms_per_step'], d['config']['launch'].get('n_splits'))" $f.json "splits=$v $c r$r"
    done
  done
done
