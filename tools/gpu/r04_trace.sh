set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04t; mkdir -p $O
for w in hotpot90k hotpot90k_d384; do
  for f in 0 0x4000000; do
    echo "== $w flags $f"
    timeout -k 10 240 python -u tools/qres_trace.py --workload $w --flags $f --json $O/${w}_$f.json > $O/${w}_$f.log 2>&1 || { echo FAIL; tail -20 $O/${w}_$f.log; exit 1; }
    tail -3 $O/${w}_$f.log
  done
done
