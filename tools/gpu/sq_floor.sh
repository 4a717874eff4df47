#!/bin/bash
# SQ counter passes of one register-resident launch kind (tools/c3_floor.py --only): self-seeded,
# perfect caller seed, GEMM-only (ablation build). usage: sq_floor.sh OUT WORKLOAD
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/sq_floor}; W=${2:-hotpot90k}; mkdir -p $O
export AHR_LIB_PATH=ah-rag_amd/ah_rag/_lib/ablation/libahr_hip.so
ST=20; [ $W == synth5m ] && ST=4
for v in self_seeded perfect gemm_only; do
  run() {  # name, counters...
    local name=$1; shift
    timeout -s KILL 150 rocprofv3 --pmc "$@" -d "$O/$v/$name" --output-format csv -- python -u tools/c3_floor.py --workload $W --only $v --steps $ST > "$O/$v/$name.log" 2>&1
  }
  mkdir -p $O/$v
  run util SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE || exit 1
  run lds SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU || exit 1
  run salu SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_INSTS_VALU || exit 1
  echo $v; python tools/sq_summary.py $O/$v --kernel topk_qres
done
