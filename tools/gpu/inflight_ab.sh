#!/bin/bash
# Two-in-flight plan checks: the wave-form pre-pass up to B = 128 (AHR_PREPASS_WAVE_B) and the
# automatic tile cap beyond two query blocks (AHR_TILE_SLOTS=256 at B = 384 / 511), alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/inflight}; mkdir -p $O
run() {  # name batch env...
  local n=$1 b=$2; shift 2
  timeout -k 10 200 env "$@" python -u bench.py --batch $b --steps 1000 --no-sublines --no-f32-line --no-batch-sweep --no-cpu-baseline > $O/$n.json 2> $O/$n.err || { echo FAIL $n; tail -5 $O/$n.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['config']['serial_ms_per_step'], d['config']['launch'].get('n_splits'), d['stages_ms_per_step'].get('threshold_prepass'))" $O/$n.json "$n"
}
for r in 1 2; do
  run b128_w64_r$r 128 AHR_PREPASS_WAVE_B=64 || exit 1
  run b128_w128_r$r 128 AHR_PREPASS_WAVE_B=128 || exit 1
  run b96_w64_r$r 96 AHR_PREPASS_WAVE_B=64 || exit 1
  run b96_w128_r$r 96 AHR_PREPASS_WAVE_B=128 || exit 1
  run b384_s512_r$r 384 AHR_TILE_SLOTS=512 || exit 1
  run b384_s256_r$r 384 AHR_TILE_SLOTS=256 || exit 1
done
