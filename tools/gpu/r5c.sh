#!/bin/bash
# Round-5 third pass: GPU tests on the current library, cooperative-compaction A/B against the
# previous build at C2 and d = 384, the seed-quality sweep (tools/seed_floor.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/r5c}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 || { echo TESTS_FAILED; tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
A=$PWD/ah-rag_amd/ah_rag/_lib/gran/libahr_hip.so
B=$PWD/ah-rag_amd/ah_rag/_lib/libahr_hip.so
for W in hotpot90k hotpot90k_d384; do bash tools/gpu/ab_lib.sh $O/ab_$W 3 $W $A $B || exit 1; done
timeout -k 10 400 python -u tools/seed_floor.py > $O/seed_floor.json 2> $O/seed_floor.err || { echo SEED_FLOOR_FAIL; tail -5 $O/seed_floor.err; exit 1; }
cat $O/seed_floor.json
