#!/bin/bash
# PMC passes over a short bench run (one counter group per pass, each under its own time limit).
# Usage (on the GPU box): bash tools/profile_pmc.sh <outdir> [bench args...]
set -u
OUT=${1:-gpurun_out/pmc}; shift || true
# --inflight 1: per-kernel durations without the deliberate cross-batch overlap (the roofline is
# per launch; bench.py takes it from a serial event-timed pass too)
ARGS=${@:-"--steps 10 --warmup 3 --no-cpu-baseline --inflight 1 --no-sublines"}
export TMPDIR=/tmp
mkdir -p "$OUT"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" --output-format csv -- python -u bench.py $ARGS > "$OUT/trace.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" --output-format csv -- python -u bench.py $ARGS > "$OUT/fetch.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" --output-format csv -- python -u bench.py $ARGS > "$OUT/write.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d "$OUT/sq" --output-format csv -- python -u bench.py $ARGS > "$OUT/sq.log" 2>&1 || exit $?
echo done
