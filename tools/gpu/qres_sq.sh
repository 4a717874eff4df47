# SQ counters of the qres forms (ablation build): p16 (full), max16 (maxima + ballot only), p32.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/qres_sq
mkdir -p $OUT
export AHR_LIB_PATH=ah-rag_amd/ah_rag/_lib/ablation/libahr_hip.so
ARGS="--batches 1024 --rounds 1 --variants p16:-1:268435456,max16:-1:268435712,p32:-1:0"
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/$name" --output-format csv -- python -u tools/dense_ablation.py $ARGS > "$OUT/$name.log" 2>&1
}
run util SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE || exit $?
run lds SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_VALU || exit $?
python tools/sq_summary.py $OUT --kernel topk_qres > $OUT/summary.jsonl
cat $OUT/summary.jsonl
