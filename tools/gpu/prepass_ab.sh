#!/bin/bash
# Threshold pre-pass wave form vs the 128 x 128 tile form (AHR_PREPASS_TILE=1), alternating on one
# box: dense parity tests, bench lines at B = 64 / 256 (bf16) and B = 64 (fp32), a kernel trace at B = 64
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/prepass}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_dense_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAIL; tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for e in "AHR_PREPASS_TILE=1" "AHR_PREPASS_TILE=0"; do
    for b in 64 128; do
      f=$O/b${b}_${e#AHR_PREPASS_TILE=}_r$r
      timeout -k 10 200 env $e python -u bench.py --batch $b --steps 1000 --no-sublines --no-f32-line --no-batch-sweep --no-cpu-baseline > $f.json 2> $f.err || { echo FAIL $e $b; tail -5 $f.err; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['config']['serial_ms_per_step'], d['config']['launch']['kernel'], d['stages_ms_per_step'], d['recall_at_10'])" $f.json "$e B=$b r$r"
    done
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace --output-format csv -- python3 -u bench.py --batch 64 --steps 200 --no-sublines --no-f32-line --no-batch-sweep --no-cpu-baseline > $O/trace_b64.json 2> $O/trace_b64.err || { echo TRACE FAIL; tail -5 $O/trace_b64.err; exit 1; }
find $O/trace -name "*kernel_stats.csv" -exec cp {} $O/b64_kernel_stats.csv \;
head -8 $O/b64_kernel_stats.csv | cut -c1-160
