set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
# kb256 at C3: GEMM only with the corpus operands from HBM (production addresses), from tile 0
# (L2-resident), from the split's first tile (MALL/L2), and with no loads after the first step
timeout -k 10 400 python -u tools/dense_ablation.py --workload synth5m --dtype f16 --batches 1024 --steps 5 --rounds 2 \
  --variants prod:-1:0,gemm_only:-1:2,gemm_tile0:-1:1048578,gemm_first:-1:2097154,gemm_noloads:-1:514 > gpurun_out/kb_l2.log 2>&1 || { tail -20 gpurun_out/kb_l2.log; exit 1; }
tail -1 gpurun_out/kb_l2.log
