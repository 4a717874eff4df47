#!/bin/bash
# cost split of the one-call drop-in search (AHR_SEARCH_SKIP bits: 1 query copy, 2 result copy, 4 rerank)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/it3}; mkdir -p $O
for sk in 0 1 2 3 7 0; do
  AHR_SEARCH_SKIP=$sk timeout -k 10 300 python -u tools/profile_single_env.py --search --raw --envs 1024 > $O/skip$sk.txt 2>&1 || { echo PROF_FAIL; tail -20 $O/skip$sk.txt; exit 1; }
  echo "skip $sk: $(grep -h 'ms per call' $O/skip$sk.txt | tr '\n' ' ')"
done
