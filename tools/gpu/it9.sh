#!/bin/bash
# environment-path tests + the single-environment rate (3 timed passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/it9}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_c5_env_gpu.py tests/test_dropin_gpu.py tests/test_lca_gpu.py tests/test_vec_env_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 || { echo TESTS_FAILED; tail -40 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
for r in 1 2; do
  timeout -k 10 200 python -u tools/profile_single_env.py --envs 128 --reps 3 > $O/single_$r.txt 2>&1 || { echo FAIL; tail -5 $O/single_$r.txt; exit 1; }
  grep "^rep" $O/single_$r.txt | tr '\n' ' '; echo
done
