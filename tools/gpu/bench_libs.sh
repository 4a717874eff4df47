#!/bin/bash
# Same-box A/B of library builds on the default C2 bench line (no sub-lines or baselines), after
# the GPU tests on the in-tree build. usage: bash tools/gpu/bench_libs.sh OUT ROUNDS "PYTEST_K" LIB...
# (PYTEST_K: a -k expression, "" = every -m gpu test, "none" = no tests; labels: the libraries'
# directory names; BENCH_ARGS: extra bench.py arguments, e.g. "--dtype f32 --batch 1 --inflight 1")
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$1; R=$2; K=$3; shift 3
mkdir -p $O
if [ "$K" != "none" ]; then
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q ${K:+-k "$K"} --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 || { echo TESTS_FAILED; tail -40 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
fi
for r in $(seq 1 $R); do for lib in "$@"; do
  v=$(basename $(dirname $lib))
  AHR_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --no-sublines --no-cpu-baseline --no-batch-sweep --no-f32-line $BENCH_ARGS > $O/bench_${v}_r$r.json 2> $O/bench_${v}_r$r.err || { echo BENCH_FAIL; tail -5 $O/bench_${v}_r$r.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['config'].get('serial_ms_per_step'), d['stages_ms_per_step'])" $O/bench_${v}_r$r.json $v
done; done
