#!/bin/bash
# The drop-in search's fused list merge: its GPU tests, then the search split with the fused path
# (default) and with the merge launch (AHR_SEARCH_FUSE=0), alternating.
# usage: fuse_ab.sh OUT ROUNDS
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/fuse}; R=${2:-2}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_dropin_gpu.py tests/test_rerank_wave_gpu.py tests/test_c5_env_gpu.py tests/test_collection_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in $(seq 1 $R); do
  for f in 1 0; do
    AHR_SEARCH_FUSE=$f timeout -k 10 300 python -u tools/search_host_split.py --n 2000 > $O/split_f${f}_r$r.txt 2>&1 || { echo SPLIT_FAILED; tail -5 $O/split_f${f}_r$r.txt; exit 1; }
    echo "fuse=$f $(tail -1 $O/split_f${f}_r$r.txt)"
  done
done
