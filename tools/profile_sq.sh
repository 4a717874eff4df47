#!/bin/bash
# SQ / TCC counter passes over a short bench run (kernel efficiency diagnosis). One pass per
# counter group, each under its own time limit. Usage (GPU box): bash tools/profile_sq.sh <outdir> [bench args]
set -u
OUT=${1:-gpurun_out/sq}; shift || true
ARGS=${@:-"--steps 10 --warmup 3 --no-cpu-baseline"}
export TMPDIR=/tmp
mkdir -p "$OUT"
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/$name" --output-format csv -- python -u bench.py $ARGS > "$OUT/$name.log" 2>&1
}
run util SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE || exit $?
run lds SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU || exit $?
run l2 TCC_HIT_sum TCC_MISS_sum || exit $?
echo done
