# C3 (5M x 768 f16, B = 1024): the register-resident kernel (default plan) vs kb256 (kFlagNoQres).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/c3_qres
timeout -k 10 300 python -u bench.py --workload synth5m --steps 10 --warmup 3 --no-cpu-baseline --no-batch-sweep > gpurun_out/c3_qres/qres.json 2> gpurun_out/c3_qres/qres.err || { tail -5 gpurun_out/c3_qres/qres.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload synth5m --steps 10 --warmup 3 --no-cpu-baseline --no-batch-sweep --debug-flags 131072 > gpurun_out/c3_qres/kb.json 2> gpurun_out/c3_qres/kb.err || { tail -5 gpurun_out/c3_qres/kb.err; exit 1; }
python - <<'PY'
import json
for n in ("qres", "kb"):
    d = json.load(open(f"gpurun_out/c3_qres/{n}.json"))
    print(n, d["value"], d["ms_per_step"], d["roofline"], d["config"].get("serial_ms_per_step"), d.get("stages_ms_per_step"), d.get("recall_at_10"))
PY
