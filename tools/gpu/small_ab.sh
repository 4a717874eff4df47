# A/B of the small-batch kernels between two builds (base = ab/libahr_hip_base.so), alternating processes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/small_ab.log
for rep in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then export AHR_LIB_PATH=$GRAFT_REPO_ROOT/ab/libahr_hip_base.so; else unset AHR_LIB_PATH; fi
    for dt in bf16 f32; do
      echo "== $v $dt" >> gpurun_out/small_ab.log
      timeout -k 10 200 python -u tools/dense_ablation.py --dtype $dt --batches 1,4 --rounds 3 --steps 50 --variants prod:-1:0 2>/dev/null | grep -v amdgpu.ids >> gpurun_out/small_ab.log || { echo FAIL; exit 1; }
    done
  done
done
python - <<'PY'
import json
cur=None
for line in open("gpurun_out/small_ab.log"):
    if line.startswith("=="): cur=line.strip(); continue
    d=json.loads(line); print(cur, d["B"], d["prod"]["tile_topk"], d["prod"]["merge"], d["prod_qps"])
PY
