# headline bench (two batches in flight) at pre-pass sample sizes, alternating processes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/sample_ab
for rep in 1 2 3; do
  for S in -1 4096 16384; do
    timeout -k 10 200 python -u bench.py --steps 400 --warmup 20 --no-cpu-baseline --no-f32-line --sample-rows $S > gpurun_out/sample_ab/s${S}_r$rep.json 2>/dev/null || { echo FAIL; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['config']['serial_ms_per_step'], d['stages_ms_per_step'])" gpurun_out/sample_ab/s${S}_r$rep.json S=$S
  done
done
