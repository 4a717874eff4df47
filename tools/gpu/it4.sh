#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/it4}; mkdir -p $O
timeout -k 10 30 ./tools/permlane_probe > $O/permlane.txt 2>&1 && cat $O/permlane.txt && timeout -k 10 600 python -u -m pytest tests/test_rerank_wave_gpu.py tests/test_rerank_rounding.py tests/test_dropin_gpu.py tests/test_collection_gpu.py tests/test_vec_env_gpu.py tests/test_c5_env_gpu.py tests/test_lca_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 || { echo TESTS_FAILED; tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
for sk in 0 4; do
  AHR_SEARCH_SKIP=$sk timeout -k 10 300 python -u tools/profile_single_env.py --search --raw --envs 1024 > $O/skip$sk.txt 2>&1 || { echo PROF_FAIL; tail -20 $O/skip$sk.txt; exit 1; }
  echo "skip $sk: $(grep -h 'ms per call' $O/skip$sk.txt | tr '\n' ' ')"
done
AHR_RERANK_SERIAL=1 timeout -k 10 300 python -u tools/profile_single_env.py --search --raw --envs 1024 > $O/serial.txt 2>&1 || { echo PROF_FAIL; exit 1; }
echo "serial rerank: $(grep -h 'ms per call' $O/serial.txt | tr '\n' ' ')"
timeout -k 10 400 python -u tools/bench_env.py --envs 1024 --episodes 3 > $O/bench_env.json 2> $O/bench_env.err || { echo ENV_FAIL; tail -20 $O/bench_env.err; exit 1; }
python - $O/bench_env.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print({k: d.get(k) for k in ("vec_env_steps_per_s", "single_env_steps_per_s", "dropin_search_b1", "reference_loop", "device_host_split_rank0")})
PY
