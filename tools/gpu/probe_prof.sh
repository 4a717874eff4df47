set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/probe_prof --output-format csv -- python -u tools/seed_probe.py --clusters 4096 --probes 2 > gpurun_out/probe_prof.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/probe_prof.log; exit 1; }
f=$(find gpurun_out/probe_prof -name "*kernel_stats.csv" | head -1)
python - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'ahr' in r['Name'] or 'Radix' in r['Name'] or 'index' in r['Name']:
        print(r['Name'][:70], r['Calls'], r['AverageNs'])
PY
