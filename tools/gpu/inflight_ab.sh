# headline bench with 2 vs 3 batches in flight, alternating processes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/inflight_ab
for rep in 1 2 3; do
  for I in 2 3; do
    timeout -k 10 200 python -u bench.py --steps 400 --warmup 20 --no-cpu-baseline --no-f32-line --inflight $I > gpurun_out/inflight_ab/i${I}_r$rep.json 2>/dev/null || { echo FAIL; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/inflight_ab/i${I}_r$rep.json inflight=$I
  done
done
