set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fold_prof --output-format csv -- python -u tools/fold_latency.py --calls 200 --rounds 1 > gpurun_out/fold_prof.log 2>&1 || { tail -20 gpurun_out/fold_prof.log; exit 1; }
f=$(find gpurun_out/fold_prof -name "*kernel_stats.csv" | head -1)
python - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'small' in r['Name'] or 'merge_block' in r['Name'] or 'convert_rows' in r['Name']:
        print(r['Name'][:70], r['Calls'], r['AverageNs'])
PY
