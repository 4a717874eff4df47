#!/bin/bash
# The drop-in / environment GPU tests, then the drop-in search host split and the C5 env line.
# usage: host_check.sh OUT
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/host}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_dropin_gpu.py tests/test_c5_env_gpu.py tests/test_vec_env_gpu.py tests/test_collection_gpu.py tests/test_lca_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/search_host_split.py --n 2000 > $O/split.txt 2>&1 || { echo SPLIT_FAILED; tail -5 $O/split.txt; exit 1; }
tail -1 $O/split.txt
timeout -k 10 400 python -u bench.py --workload env > $O/env.json 2> $O/env.err || { echo ENV_FAILED; tail -5 $O/env.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); c=d.get('c5_env') or d.get('c5') or d; print({k: c.get(k) for k in ('vec_env_steps_per_s','single_env_steps_per_s','single_env_passes','dropin_search_b1')})" $O/env.json
