#!/bin/bash
# Round-5 second pass: GPU tests, qres granule/short-list A/B (previous vs current library) at C2
# and d = 384, PMC of the current C2 kernel, small-kernel split A/B, the default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/r5b}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 || { echo TESTS_FAILED; tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
BASE=$PWD/ah-rag_amd/ah_rag/_lib/base/libahr_hip.so
NEW=$PWD/ah-rag_amd/ah_rag/_lib/libahr_hip.so
for W in hotpot90k hotpot90k_d384; do bash tools/gpu/ab_lib.sh $O/ab_$W 3 $W $BASE $NEW || exit 1; done
for r in 1 2; do for sp in 256 512; do
  AHR_SMALL_SPLITS=$sp timeout -k 10 200 python -u tools/small_ab.py --batches 1,4 > $O/small_s${sp}_r$r.json 2> $O/small_s${sp}_r$r.err || { echo SMALL_FAIL; tail -5 $O/small_s${sp}_r$r.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], {k: (v['warm_us']['tile_topk'], v['cold_us']['tile_topk'], v['cold_dirty_us']['tile_topk']) for k, v in d.items() if k != 'lib'})" $O/small_s${sp}_r$r.json $sp
done; done
timeout -k 10 300 python -u tools/seed_floor.py > $O/seed_floor.json 2> $O/seed_floor.err || { echo SEED_FLOOR_FAIL; tail -5 $O/seed_floor.err; exit 1; }
cat $O/seed_floor.json
bash tools/gpu/profile.sh $O/final_c2 hotpot90k || exit 1
timeout -k 10 400 python -u bench.py > $O/bench_n1.json 2> $O/bench_n1.err || { echo BENCH_FAIL; tail -20 $O/bench_n1.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('C2', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac']); print('d384', d['hotpot90k_d384']['roofline']['avg_launch_ms'], d['hotpot90k_d384']['roofline']['frac']); print('b1', d['batch_sweep'][0]['roofline_cold_caches']); print('f32b1', d['exact_fp32'].get('batch1'))" $O/bench_n1.json
