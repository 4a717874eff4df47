set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04b
timeout -k 10 300 python -u -m pytest tests/test_qres_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r04b/qres_tests.log 2>&1 || { echo QRES_TESTS_FAILED; tail -30 gpurun_out/r04b/qres_tests.log; exit 1; }
tail -2 gpurun_out/r04b/qres_tests.log
bash tools/gpu/ab_bench.sh gpurun_out/r04b/ab 2 "--debug-flags 0" "--debug-flags 268435456" "--debug-flags 134217728" "--debug-flags 67108864" "--debug-flags 335544320" "AHR_LIB_PATH=ah-rag_amd/ah_rag/_lib/r03/libahr_hip.so@--debug-flags 0" -- --steps 200 --warmup 20
bash tools/gpu/ab_bench.sh gpurun_out/r04b/c3 1 "--debug-flags 0" "--debug-flags 8388608" -- --workload synth5m --steps 10 --warmup 2
timeout -k 10 400 python -u bench.py > gpurun_out/r04b/bench_default.json 2> gpurun_out/r04b/bench_default.err || { echo BENCH_DEFAULT_FAIL; tail -20 gpurun_out/r04b/bench_default.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r04b/bench_default.json"))
print("C2", d["value"], d["ms_per_step"], d["config"]["serial_ms_per_step"], d["roofline"]["avg_launch_ms"], d["roofline"]["frac"], d["config"]["threshold_seed"][:30])
for key in ("synth5m", "hotpot90k_d384", "c5_env"):
    s = d.get(key) or {}
    print(key, {k: s.get(k) for k in ("value", "ms_per_step", "recall_at_10", "vec_env_steps_per_s", "single_env_steps_per_s", "launch")}, (s.get("roofline") or {}).get("frac"))
print("b1", [(b["batch"], b["value"], b["roofline"]["frac"], (b.get("roofline_cold_caches") or {}).get("frac")) for b in d.get("batch_sweep", [])])
PY
