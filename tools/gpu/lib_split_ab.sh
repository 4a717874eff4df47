#!/bin/bash
# The drop-in search's host split (tools/search_host_split.py) with two library builds, alternating,
# after the drop-in / rerank / env GPU tests on the in-tree build.
# usage: lib_split_ab.sh OUT ROUNDS LIB_A LIB_B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$1; R=$2; A=$3; B=$4; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_dropin_gpu.py tests/test_rerank_wave_gpu.py tests/test_c5_env_gpu.py tests/test_collection_gpu.py tests/test_vec_env_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in $(seq 1 $R); do
  for v in A B; do
    lib=$A; [ $v == B ] && lib=$B
    AHR_LIB_PATH=$lib timeout -k 10 300 python -u tools/search_host_split.py --n 2000 > $O/split_${v}_r$r.txt 2>&1 || { echo SPLIT_FAILED; tail -5 $O/split_${v}_r$r.txt; exit 1; }
    python -c "
import ast,sys; d=ast.literal_eval(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['native_call'], d['search_batch'], d['engine.run(numpy, borrow)'])" $O/split_${v}_r$r.txt $v
  done
done
