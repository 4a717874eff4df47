#!/bin/bash
# Full GPU check on one box: every -m gpu test, smoke(), the default bench line.
# usage: bash tools/gpu/check.sh [OUTDIR] [extra pytest args]   (e.g. AHR_PARITY_LOG=... to keep margins)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/check}; shift || true
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread "$@" > $O/gputests.log 2>&1 || { echo TESTS_FAILED; tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_n1.json 2> $O/bench_n1.err || { echo BENCH_FAIL; tail -20 $O/bench_n1.err; exit 1; }
python - $O/bench_n1.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("C2", d["value"], d["ms_per_step"], d["config"]["serial_ms_per_step"], d["roofline"]["avg_launch_ms"], d["roofline"]["frac"])
for key in ("synth5m", "c5_env"):
    s = d.get(key) or {}
    print(key, {k: s.get(k) for k in ("value", "ms_per_step", "recall_at_10", "vec_env_steps_per_s", "single_env_steps_per_s")},
          (s.get("roofline") or {}).get("frac"))
PY
