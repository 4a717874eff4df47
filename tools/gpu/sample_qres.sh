# C2 with the register-resident kernel: pre-pass sample size S vs end-to-end (serial and inflight).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/sample_qres
for S in 4096 8192 16384; do
timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-batch-sweep --no-f32-line --sample-rows $S > gpurun_out/sample_qres/s$S.json 2> gpurun_out/sample_qres/s$S.err || { tail -5 gpurun_out/sample_qres/s$S.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/sample_qres/s$S.json')); print($S, d['value'], d['ms_per_step'], d['config']['serial_ms_per_step'], d['stages_ms_per_step'])"
done
