#!/bin/bash
# Environment / drop-in GPU tests, then the single-environment profile and the C5 line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/env_check}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_vec_env_gpu.py tests/test_c5_env_gpu.py tests/test_dropin_gpu.py tests/test_rerank_rounding.py tests/test_lca_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python -u tools/profile_single_env.py > $O/single_prof.txt 2>&1 || { echo PROF_FAILED; tail -20 $O/single_prof.txt; exit 1; }
grep "single env" $O/single_prof.txt
timeout -k 10 400 python -u bench.py --workload env --no-cpu-baseline > $O/bench_env.json 2> $O/bench_env.err || { echo BENCH_FAILED; tail -20 $O/bench_env.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print({k: d.get(k) for k in ('value','unit')}, d.get('single_env_steps_per_s'), d.get('vec_env_steps_per_s'))" $O/bench_env.json
