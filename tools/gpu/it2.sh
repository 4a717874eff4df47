#!/bin/bash
# host-path profile of the drop-in search / single env, and qres vs tilelane at small batches
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/it2}; mkdir -p $O
timeout -k 10 300 python -u tools/profile_single_env.py --search --raw --envs 512 > $O/prof_search.txt 2>&1 || { echo PROF_FAIL; tail -20 $O/prof_search.txt; exit 1; }
head -4 $O/prof_search.txt
timeout -k 10 300 python -u tools/profile_single_env.py --envs 128 > $O/prof_single.txt 2>&1 || { echo PROF_FAIL; tail -20 $O/prof_single.txt; exit 1; }
head -2 $O/prof_single.txt
for b in 64 128 256; do
  for f in 0 8388608; do
    timeout -k 10 200 python -u bench.py --batch $b --steps 400 --clock-ramp 200 --no-sublines --no-f32-line --no-batch-sweep --no-cpu-baseline --debug-flags $f > $O/b${b}_f$f.json 2> $O/b${b}_f$f.err || { echo BENCH_FAIL $b $f; tail -5 $O/b${b}_f$f.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/b${b}_f$f.json')); print($b, $f, d['value'], d['ms_per_step'], d['config']['launch'], d['stages_ms_per_step'], d['recall_at_10'])"
  done
done
