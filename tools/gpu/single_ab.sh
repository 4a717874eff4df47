#!/bin/bash
# single-environment A/B on one box: the small expansion path and the node-brief cache, alternated
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/single_ab}; mkdir -p $O
for r in 1 2; do
  timeout -k 10 200 python -u tools/profile_single_env.py --envs 128 --reps 3 > $O/default_$r.txt 2>&1 || { echo FAIL; tail -5 $O/default_$r.txt; exit 1; }
  grep "^rep\|single env" $O/default_$r.txt | tr '\n' ' '; echo " <- default"
  AHR_EXPAND_SMALL=0 timeout -k 10 200 python -u tools/profile_single_env.py --envs 128 --reps 3 > $O/nosmall_$r.txt 2>&1 || { echo FAIL; tail -5 $O/nosmall_$r.txt; exit 1; }
  grep "^rep\|single env" $O/nosmall_$r.txt | tr '\n' ' '; echo " <- AHR_EXPAND_SMALL=0"
  timeout -k 10 200 python -u tools/profile_single_env.py --envs 128 --reps 3 --no-brief-cache > $O/nocache_$r.txt 2>&1 || { echo FAIL; tail -5 $O/nocache_$r.txt; exit 1; }
  grep "^rep\|single env" $O/nocache_$r.txt | tr '\n' ' '; echo " <- no brief cache"
done
