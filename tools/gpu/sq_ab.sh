set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in tl_full:0 tl_gemm:34 kb_full:524288 kb_gemm:524290; do
  name=${cfg%%:*}; fl=${cfg##*:}
  bash tools/profile_sq.sh gpurun_out/sq_$name --steps 10 --warmup 3 --no-cpu-baseline --inflight 1 --debug-flags $fl || { echo "PROFILE FAILED $name"; exit 1; }
  python tools/sq_summary.py gpurun_out/sq_$name > gpurun_out/sq_$name.json
done
for f in gpurun_out/sq_*.json; do echo "== $f"; cat $f; done
