set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04abl; mkdir -p $O
export AHR_LIB_PATH=ah-rag_amd/ah_rag/_lib/ablation/libahr_hip.so
V="prod:-1:0,prepass:-1:67108864,gemm:-1:2,gemm_noloads:-1:514,gemm_nowait:-1:1026,gemm_nowait_nobar:-1:16778242,gemm_noread:-1:33554434,gemm_all:-1:50333186"
for w in hotpot90k hotpot90k_d384; do
  timeout -k 10 300 python -u tools/dense_ablation.py --workload $w --batches 1024 --steps 30 --rounds 3 --variants $V > $O/$w.log 2>&1 || { echo FAIL; tail -20 $O/$w.log; exit 1; }
  python - $O/$w.log <<'P'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l)
        for k,v in d.items():
            if isinstance(v,dict) and 'tile_topk' in v: print(sys.argv[1].split('/')[-1], f"{k:20s} tile {v['tile_topk']*1000:.1f} us  total {sum(v.values())*1000:.1f}")
P
done
