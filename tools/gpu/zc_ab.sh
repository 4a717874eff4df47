#!/bin/bash
# The drop-in search writing its results straight into the pinned host buffer: its GPU tests, then
# the search split with it (default) and with the result copy (AHR_SEARCH_ZC=0), alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/zc}; R=${2:-2}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_dropin_gpu.py tests/test_rerank_wave_gpu.py tests/test_c5_env_gpu.py tests/test_collection_gpu.py tests/test_vec_env_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in $(seq 1 $R); do
  for f in 1 0; do
    AHR_SEARCH_ZC=$f timeout -k 10 300 python -u tools/search_host_split.py --n 2000 > $O/split_zc${f}_r$r.txt 2>&1 || { echo SPLIT_FAILED; tail -5 $O/split_zc${f}_r$r.txt; exit 1; }
    echo "zc=$f $(tail -1 $O/split_zc${f}_r$r.txt | cut -c1-200)"
  done
done
