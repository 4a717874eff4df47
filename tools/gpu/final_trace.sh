# Round-3 closing evidence on ONE box: the default bench line, then the rocprofv3 kernel-trace
# stats of the same workload (single batch in flight), so the two kernel times can be compared.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/final_trace
mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench_n1.json 2> $O/bench_n1.err || { echo BENCH_FAIL; tail -20 $O/bench_n1.err; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/trace --output-format csv -- python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --inflight 1 --no-batch-sweep --no-f32-line > $O/trace.log 2>&1 || { echo TRACE_FAIL; tail -20 $O/trace.log; exit 1; }
python - <<'PY'
import csv, glob, json
d = json.load(open("gpurun_out/final_trace/bench_n1.json"))
print("bench", d["value"], d["roofline"]["avg_launch_ms"], d["config"]["serial_ms_per_step"])
t = [json.loads(l) for l in open("gpurun_out/final_trace/trace.log") if l.startswith('{"metric"')][0]
print("bench under trace", t["value"], t["roofline"]["avg_launch_ms"])
f = glob.glob("gpurun_out/final_trace/trace/*/*kernel_stats.csv")[0]
for r in csv.DictReader(open(f)):
    if "ahr::" in r["Name"]:
        print(r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), r["Name"][:70])
PY
