#!/bin/bash
# single-environment latency pass: expansion tests, bench_env, cProfile of the single env loop
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/it8}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_lca_gpu.py tests/test_c5_env_gpu.py tests/test_vec_env_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 || { echo TESTS_FAILED; tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
timeout -k 10 400 python -u tools/bench_env.py --envs 1024 --episodes 3 > $O/bench_env.json 2> $O/bench_env.err || { echo ENV_FAIL; tail -20 $O/bench_env.err; exit 1; }
python - $O/bench_env.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print({k: d.get(k) for k in ("vec_env_steps_per_s", "single_env_steps_per_s", "reference_loop_steps_per_s", "dropin_search_b1", "vec_step_ms_rank0")})
PY
timeout -k 10 300 python -u tools/profile_single_env.py --envs 64 > $O/profile_single.txt 2>&1 || { echo PROF_FAIL; tail -5 $O/profile_single.txt; exit 1; }
head -45 $O/profile_single.txt
