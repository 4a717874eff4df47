set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for P in 2; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/probe_p$P --output-format csv -- python -u tools/seed_probe.py --clusters 4096 --probes 2 --probe-clusters $P > gpurun_out/probe_p$P.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/probe_p$P.log; exit 1; }
grep -o '"device_production_ms_per_batch.*' gpurun_out/probe_p$P.log | cut -c1-400
f=$(find gpurun_out/probe_p$P -name "*kernel_stats.csv" | head -1)
python - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'probe_seed' in r['Name'] or 'tilelane_kernel<2, 8>' in r['Name'] or 'merge_lane_lists_kernel<8>' in r['Name']:
        print(r['Name'][:60], r['Calls'], r['AverageNs'])
PY
done
