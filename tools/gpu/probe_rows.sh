set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/probe_rows.py --per-cluster 50,100,200 > gpurun_out/probe_rows.log 2>&1 || { tail -20 gpurun_out/probe_rows.log; exit 1; }
cat gpurun_out/probe_rows.log | grep rows
