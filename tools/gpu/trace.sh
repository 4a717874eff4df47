#!/bin/bash
# The default bench line, then the rocprofv3 kernel-trace stats of the same workload (one batch in
# flight, no sub-lines) on ONE box, so the two kernel times can be compared.
# usage: bash tools/gpu/trace.sh [OUTDIR] [extra bench args for both runs]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/trace}; shift || true
mkdir -p $O
timeout -k 10 400 python -u bench.py "$@" > $O/bench_n1.json 2> $O/bench_n1.err || { echo BENCH_FAIL; tail -20 $O/bench_n1.err; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/trace --output-format csv -- python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --inflight 1 --no-batch-sweep --no-f32-line --no-sublines "$@" > $O/trace.log 2>&1 || { echo TRACE_FAIL; tail -20 $O/trace.log; exit 1; }
python - $O <<'PY'
import csv, glob, json, sys
o = sys.argv[1]
d = json.load(open(f"{o}/bench_n1.json"))
print("bench", d["value"], d["roofline"]["avg_launch_ms"], d["config"]["serial_ms_per_step"])
t = [json.loads(l) for l in open(f"{o}/trace.log") if l.startswith('{"metric"')][0]
print("bench under trace", t["value"], t["roofline"]["avg_launch_ms"])
f = glob.glob(f"{o}/trace/*/*kernel_stats.csv")[0]
for r in csv.DictReader(open(f)):
    if "ahr::" in r["Name"]:
        print(r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), r["Name"][:70])
PY
