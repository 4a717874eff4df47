set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for v in prod probe; do
    extra=""; [ $v = probe ] && extra="--probe-seeds"
    timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-f32-line $extra > gpurun_out/pb_$v.json 2> gpurun_out/pb_$v.err || { echo BENCH_FAIL $v; tail -20 gpurun_out/pb_$v.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/pb_$v.json')); print('$v', d['value'], d['ms_per_step'], d['config']['serial_ms_per_step'], d['stages_ms_per_step'], d['roofline']['frac'], d['recall_at_10'], d['config']['threshold_seed'])"
  done
done
