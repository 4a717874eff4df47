set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/probe_c3
# C3 (5M x 768 f16, B = 1024): production (sampled pre-pass) vs cluster-probe seeds at two cluster counts
timeout -k 10 300 python -u bench.py --workload synth5m --steps 10 --warmup 3 > gpurun_out/probe_c3/prod.json 2> gpurun_out/probe_c3/prod.err || { tail -5 gpurun_out/probe_c3/prod.err; exit 1; }
for C in 25000 50000; do
timeout -k 10 400 python -u bench.py --workload synth5m --steps 10 --warmup 3 --probe-seeds --probe-clusters $C > gpurun_out/probe_c3/probe_$C.json 2> gpurun_out/probe_c3/probe_$C.err || { tail -5 gpurun_out/probe_c3/probe_$C.err; exit 1; }
done
python - <<'PY'
import json
for n in ("prod", "probe_25000", "probe_50000"):
    d = json.load(open(f"gpurun_out/probe_c3/{n}.json"))
    print(n, d["value"], d["ms_per_step"], d["roofline"]["frac"], d["config"].get("serial_ms_per_step"), d["stages_ms_per_step"], d["config"].get("threshold_seed"), d.get("recall_at_10"))
PY
