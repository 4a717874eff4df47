#!/bin/bash
# Round-5 first GPU pass: full check, small-kernel A/B (previous vs current library), qres cost
# split at d = 768 / 384 (ablation build), d = 384 PMC passes, clock-ramp A/B. (For this pass the
# ablation library was copied to _lib/abl/: _lib/ablation/ is in .gpurunignore.)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/r5a}
mkdir -p $O
AHR_PARITY_LOG=$O/check/parity_margins.jsonl bash tools/gpu/check.sh $O/check || exit 1
for r in 1 2; do
  for v in base new; do
    lib=ah-rag_amd/ah_rag/_lib/libahr_hip.so; [ $v == base ] && lib=ah-rag_amd/ah_rag/_lib/base/libahr_hip.so
    AHR_LIB_PATH=$PWD/$lib timeout -k 10 200 python -u tools/small_ab.py > $O/small_${v}_r$r.json 2> $O/small_${v}_r$r.err || { echo SMALL_AB_FAIL; tail -5 $O/small_${v}_r$r.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], {k: (v['warm_us']['tile_topk'], v['cold_us']['tile_topk']) for k, v in d.items() if k != 'lib'})" $O/small_${v}_r$r.json $v
  done
done
V="prod:-1:0,noscreen:-1:2,noloads:-1:512,nobarrier:-1:16777216,noread:-1:33554432,nowait_nobar:-1:17826816,gemm_noloads:-1:514,gemm_core:-1:50333186"
for W in hotpot90k hotpot90k_d384; do
  AHR_LIB_PATH=$PWD/ah-rag_amd/ah_rag/_lib/abl/libahr_hip.so timeout -k 10 300 python -u tools/dense_ablation.py --workload $W --batches 1024 --rounds 3 --variants $V > $O/abl_$W.json 2> $O/abl_$W.err || { echo ABL_FAIL; tail -5 $O/abl_$W.err; exit 1; }
  tail -1 $O/abl_$W.json | cut -c1-1500
done
bash tools/gpu/profile.sh $O/final_d384 hotpot90k_d384 || exit 1
for r in 1 2; do for ramp in 0 200; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --clock-ramp $ramp --no-sublines --no-cpu-baseline --no-batch-sweep --no-f32-line > $O/ramp${ramp}_r$r.json 2>/dev/null || exit 1
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],d['value'],d['roofline']['avg_launch_ms'])" $O/ramp${ramp}_r$r.json
done; done
