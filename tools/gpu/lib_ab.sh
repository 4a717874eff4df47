# A/B of two builds of libahr_hip.so on one box: alternating processes (base = ab/libahr_hip_base.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/lib_ab.log
for rep in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then export AHR_LIB_PATH=$GRAFT_REPO_ROOT/ab/libahr_hip_base.so; else unset AHR_LIB_PATH; fi
    echo "== $v C2" >> gpurun_out/lib_ab.log
    timeout -k 10 200 python -u tools/dense_ablation.py --batches 1024 --rounds 3 --variants prod:-1:0 2>/dev/null | grep -v amdgpu.ids >> gpurun_out/lib_ab.log || { echo FAIL; exit 1; }
    [ -n "${AB_C3:-}" ] || continue
    echo "== $v C3" >> gpurun_out/lib_ab.log
    timeout -k 10 300 python -u tools/dense_ablation.py --workload synth5m --dtype f16 --batches 1024 --rounds 2 --steps 5 --variants prod:-1:0 2>/dev/null | grep -v amdgpu.ids >> gpurun_out/lib_ab.log || { echo FAIL; exit 1; }
  done
done
python - <<'PY'
import json
cur=None
for line in open("gpurun_out/lib_ab.log"):
    if line.startswith("=="): cur=line.strip(); continue
    d=json.loads(line); print(cur, d["prod"]["tile_topk"], d["prod"]["threshold_prepass"])
PY
