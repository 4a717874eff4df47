#!/bin/bash
# Round-5 sixth pass: GPU tests on the current library (fragment copy straight from fp32), then the
# default bench line with the previous library and the current one, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/r5f}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 || { echo TESTS_FAILED; tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
L=$PWD/ah-rag_amd/ah_rag/_lib
for r in 1 2 3; do for v in base2 new; do
  lib=$L/libahr_hip.so; [ $v == base2 ] && lib=$L/base2/libahr_hip.so
  AHR_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --no-sublines --no-cpu-baseline --no-batch-sweep --no-f32-line > $O/bench_${v}_r$r.json 2> $O/bench_${v}_r$r.err || { echo BENCH_FAIL; tail -5 $O/bench_${v}_r$r.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['stages_ms_per_step'])" $O/bench_${v}_r$r.json $v
done; done
