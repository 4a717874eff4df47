#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5p
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 || { echo TESTS_FAILED; tail -40 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
timeout -k 10 400 python -u tools/profile_single_env.py --search --envs 256 > $O/search_prof.txt 2>&1 || { echo PROF_FAILED; tail -20 $O/search_prof.txt; exit 1; }
grep "search_batch" $O/search_prof.txt
timeout -k 10 400 python -u bench.py --workload env --no-cpu-baseline > $O/bench_env.json 2> $O/bench_env.err || { echo BENCH_FAILED; tail -20 $O/bench_env.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1]))['c5']; print(d['vec_env_steps_per_s'], d['single_env_steps_per_s'], d['dropin_search_b1'])" $O/bench_env.json
