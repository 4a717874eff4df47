#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/it6}; mkdir -p $O
bash tools/gpu/bench_libs.sh $O/c2 1 "" ah-rag_amd/ah_rag/_lib/libahr_hip.so ah-rag_amd/ah_rag/_lib/variant_mma32/libahr_hip.so || exit 1
BENCH_ARGS="--workload hotpot90k_d384" bash tools/gpu/bench_libs.sh $O/d384 1 none ah-rag_amd/ah_rag/_lib/libahr_hip.so ah-rag_amd/ah_rag/_lib/variant_mma32/libahr_hip.so || exit 1
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
