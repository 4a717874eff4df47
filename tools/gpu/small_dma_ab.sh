#!/bin/bash
# (the non-default forms are in the ablation build: copy ah-rag_amd/ah_rag/_lib/ablation to a
# gpurun-visible directory, e.g. _lib/abl, and export AHR_LIB_PATH=<that>/libahr_hip.so first)
# bf16 small kernel: register loads vs LDS-DMA items (AHR_SMALL_DMA), parity under the DMA form,
# kernel stage (serial, warm / cold) and bench lines at B = 1 and 16 (default in-flight count).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/small_dma}
mkdir -p $O
AHR_SMALL_DMA=1 timeout -k 10 300 python -u -m pytest tests/test_dense_gpu.py tests/test_configs_gpu.py -m gpu -x -q -k "small or b1 or bf16" --timeout 120 --timeout-method thread > $O/tests_dma.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/tests_dma.log; exit 1; }
tail -1 $O/tests_dma.log
for r in 1 2; do for v in 0 1; do
  AHR_SMALL_DMA=$v timeout -k 10 300 python -u tools/small_ab.py --batches 1,4,16 --reps 100 > $O/ab_dma${v}_r$r.json 2> $O/ab_dma${v}_r$r.err || { echo AB_FAIL; tail -5 $O/ab_dma${v}_r$r.err; exit 1; }
  python -c "
import json,sys; d=json.load(open(sys.argv[1]))
print(sys.argv[2], *[(b, d[b]['warm_us'].get('tile_topk'), d[b]['cold_us'].get('tile_topk')) for b in ('bf16_b1','bf16_b4','bf16_b16')])" $O/ab_dma${v}_r$r.json "dma$v"
done; done
bash tools/gpu/ab_bench.sh $O/b1 2 "AHR_SMALL_DMA=0@--batch 1" "AHR_SMALL_DMA=1@--batch 1" || exit 1
bash tools/gpu/ab_bench.sh $O/b16 2 "AHR_SMALL_DMA=0@--batch 16" "AHR_SMALL_DMA=1@--batch 16" || exit 1
