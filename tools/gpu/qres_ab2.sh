# Same-box A/B of the register-resident kernel: staggered waves (default) vs lock-step vs the tile
# kernel, production build; cost split of both forms (ablation build); instruction counters.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/dense_ablation.py --batches 1024 --rounds 3 --variants prod:-1:0,lockstep:-1:67108864,tl:-1:32 \
  > gpurun_out/qres_ab2.log 2>&1 || { echo AB_FAILED; tail -30 gpurun_out/qres_ab2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/qres_ab2.log | tail -1
AHR_LIB_PATH=ah-rag_amd/ah_rag/_lib/ablation/libahr_hip.so timeout -k 10 400 python -u tools/dense_ablation.py --batches 1024 --rounds 3 \
  --variants prod:-1:0,prod_ls:-1:67108864,gemm:-1:2,gemm_ls:-1:67108866,noread:-1:33554434,noread_ls:-1:100663298,bare:-1:50333186,bare_ls:-1:117442050 \
  > gpurun_out/qres_ablation2.log 2>&1 || { echo ABL_FAILED; tail -30 gpurun_out/qres_ablation2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/qres_ablation2.log | tail -1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_VALU_MFMA_COEXEC_CYCLES -d gpurun_out/qres_sq2/inst --output-format csv -- python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-f32-line --no-batch-sweep --inflight 1 > gpurun_out/qres_sq2_inst.log 2>&1 || { echo SQ_FAILED; tail -20 gpurun_out/qres_sq2_inst.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_VALU_MFMA_COEXEC_CYCLES -d gpurun_out/qres_sq2/inst_tl --output-format csv -- python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-f32-line --no-batch-sweep --inflight 1 --debug-flags 32 > gpurun_out/qres_sq2_inst_tl.log 2>&1 || { echo SQ_FAILED; tail -20 gpurun_out/qres_sq2_inst_tl.log; exit 1; }
python tools/sq_summary.py gpurun_out/qres_sq2 --kernel topk_
