# Planner check at larger batches (C2 corpus): qres256 (default) vs the plan without the
# query-resident kernels (flag 2048).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/dense_ablation.py --batches 512,2048,4096,8192 --rounds 2 --steps 10 \
  --variants qres:-1:0,noqres:-1:2048 > gpurun_out/qres_batches.log 2>&1 || { echo FAILED; tail -30 gpurun_out/qres_batches.log; exit 1; }
grep -v amdgpu.ids gpurun_out/qres_batches.log | python -c "
import json, sys
for l in sys.stdin:
    if not l.startswith('{'): continue
    d = json.loads(l)
    print(d['B'], d['plan']['kernel'], {k: (v['tile_topk'], d.get(k + '_qps')) for k, v in d.items() if isinstance(v, dict) and 'tile_topk' in v})
"
