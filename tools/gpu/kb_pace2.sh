# kb256 split pacing (asynchronous sibling poll) lead sweep at C3 (AHR_KB_PACE_LEAD, 0 = off): time and FETCH_SIZE per lead.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/kb_pace3
mkdir -p $O
A="--workload synth5m --steps 10 --warmup 3 --no-cpu-baseline --no-batch-sweep --no-f32-line"
B="--workload synth5m --steps 3 --warmup 1 --no-cpu-baseline --no-batch-sweep --no-f32-line --inflight 1"
for L in 0 12 8 0 12; do
AHR_KB_PACE_LEAD=$L timeout -k 10 300 python -u bench.py $A > $O/l$L.json 2> $O/l$L.err || { tail -5 $O/l$L.err; exit 1; }
AHR_KB_PACE_LEAD=$L timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_l$L --output-format csv -- python -u bench.py $B > $O/fetch_l$L.log 2>&1 || exit 1
python - <<PY
import csv, glob, json
d = json.load(open("$O/l$L.json"))
f = glob.glob("$O/fetch_l$L/*/*counter_collection.csv")[0]
v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "topk_kb256" in r["Kernel_Name"]]
print("lead $L", d["value"], d["roofline"]["avg_launch_ms"], "GB/launch", round(sum(v) / len(v) * 2048 / 1e9, 3))
PY
done
