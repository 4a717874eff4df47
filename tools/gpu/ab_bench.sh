#!/bin/bash
# A/B bench on one box: alternate `python bench.py` runs over flag sets, N rounds each.
# usage: tools/gpu/ab_bench.sh OUTDIR ROUNDS "VARIANT_A" "VARIANT_B" ... -- extra bench args
# a variant is bench args, optionally prefixed by environment settings and '@':
# e.g.   tools/gpu/ab_bench.sh gpurun_out/ab 2 "--debug-flags 0" "AHR_LIB_PATH=lib/old.so@--debug-flags 0" -- --inflight 1
set -o pipefail
out=$1; rounds=$2; shift 2
variants=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do variants+=("$1"); shift; done
[ "$1" == "--" ] && shift
extra=("$@")
mkdir -p "$out"
for r in $(seq 1 "$rounds"); do
  for i in "${!variants[@]}"; do
    v=${variants[$i]}
    envs=""; args=$v
    if [[ "$v" == *@* ]]; then envs=${v%%@*}; args=${v#*@}; fi
    echo "== round $r variant $i: $v ${extra[*]}"
    timeout -k 10 240 env $envs python -u bench.py --no-cpu-baseline --no-f32-line --no-batch-sweep --no-sublines $args "${extra[@]}" \
      > "$out/v${i}_r${r}.json" 2> "$out/v${i}_r${r}.err" || { echo "BENCH FAILED ($v)"; tail -5 "$out/v${i}_r${r}.err"; exit 1; }
    python - "$out/v${i}_r${r}.json" <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][0]
d = json.loads(line)
st = d.get("stages_ms_per_step", {})
print(f"  value {d['value']:.0f} ms/step {d['ms_per_step']:.4f} serial {d.get('config', {}).get('serial_ms_per_step')} "
      f"kernel_ms {d.get('roofline', {}).get('avg_launch_ms')} frac {d.get('roofline', {}).get('frac')} recall {d.get('recall_at_10')} stages {st}")
PY
  done
done
