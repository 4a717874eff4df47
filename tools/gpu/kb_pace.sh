# kb256 split pacing at C3: parity (kb256 + C3/C4 tests), then time and FETCH_SIZE with and without it.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/kb_pace
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_dense_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread -k "kb256 or kb128 or c3 or c4 or concurrent" > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
A="--workload synth5m --steps 10 --warmup 3 --no-cpu-baseline --no-batch-sweep --no-f32-line"
timeout -k 10 300 python -u bench.py $A > $O/pace.json 2> $O/pace.err || { tail -5 $O/pace.err; exit 1; }
timeout -k 10 300 python -u bench.py $A --debug-flags 1073741824 > $O/nopace.json 2> $O/nopace.err || { tail -5 $O/nopace.err; exit 1; }
python -c "
import json
for n in ('pace','nopace'):
    d=json.load(open('$O/'+n+'.json')); print(n, d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['config']['launch'])
"
B="--workload synth5m --steps 3 --warmup 1 --no-cpu-baseline --no-batch-sweep --no-f32-line --inflight 1"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_pace --output-format csv -- python -u bench.py $B > $O/fetch_pace.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_nopace --output-format csv -- python -u bench.py $B --debug-flags 1073741824 > $O/fetch_nopace.log 2>&1 || exit 1
python - <<'PY'
import csv, glob
for n in ("fetch_pace", "fetch_nopace"):
    f = glob.glob(f"gpurun_out/kb_pace/{n}/*/*counter_collection.csv")[0]
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "topk_kb256" in r["Kernel_Name"]]
    print(n, len(v), "GB per launch (x2 wide-read correction):", round(sum(v) / len(v) * 1024 * 2 / 1e9, 3))
PY
