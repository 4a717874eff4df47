#!/bin/bash
# (the non-default forms are in the ablation build: copy ah-rag_amd/ah_rag/_lib/ablation to a
# gpurun-visible directory, e.g. _lib/abl, and export AHR_LIB_PATH=<that>/libahr_hip.so first)
# fp32 small kernel A/B (B = 1 and 4, C2 corpus): load form AHR_F32_SLOTS (0 = per-lane register
# loads, 2 = LDS-DMA whole lines) x split count AHR_F32_WPS (1 = 256 workgroups, 8 = ceil(items / 8)),
# after the fp32 parity tests under each load form. usage: bash tools/gpu/f32_ab.sh gpurun_out/<dir>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/f32_ab}
mkdir -p $O
for sl in 0 2; do
AHR_F32_SLOTS=$sl timeout -k 10 300 python -u -m pytest tests/test_dense_gpu.py tests/test_configs_gpu.py -m gpu -x -q -k "f32" --timeout 120 --timeout-method thread > $O/f32tests_s$sl.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/f32tests_s$sl.log; exit 1; }
tail -1 $O/f32tests_s$sl.log
done
for r in 1 2; do for v in "0 8" "0 1" "2 1" "2 8"; do
  set -- $v; sl=$1
  AHR_F32_SLOTS=$1 AHR_F32_WPS=$2 timeout -k 10 300 python -u tools/small_ab.py --batches 1,4 --reps 100 > $O/ab_s$1_w$2_r$r.json 2> $O/ab_s$1_w$2_r$r.err || { echo AB_FAIL; tail -5 $O/ab_s$1_w$2_r$r.err; exit 1; }
  python -c "
import json,sys; d=json.load(open(sys.argv[1]))
print(sys.argv[2], *[(b, d[b]['warm_us'].get('tile_topk'), d[b]['cold_us'].get('tile_topk')) for b in ('f32_b1','f32_b4')])" $O/ab_s$1_w$2_r$r.json "slots$1 wps$2"
done; done
