set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04t2; mkdir -p $O
run() { # name workload [env...]
  n=$1; w=$2; shift 2
  echo "== $n"
  env "$@" timeout -k 10 240 python -u tools/qres_trace.py --workload $w --reps 2 --json $O/$n.json > $O/$n.log 2>&1 || { echo FAIL; tail -20 $O/$n.log; exit 1; }
  tail -1 $O/$n.log
}
run c2_default hotpot90k AHR_X=0
run c2_every hotpot90k AHR_QRES_PUB=ffffffff AHR_QRES_EV=fffffffc
run d384_default hotpot90k_d384 AHR_X=0
