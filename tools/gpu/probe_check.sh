set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_probe_seed_gpu.py > gpurun_out/probe_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/probe_tests.log; exit 1; }
tail -2 gpurun_out/probe_tests.log
timeout -k 10 400 python -u tools/seed_probe.py --clusters 4096 --probes 2 --batch 1024 > gpurun_out/seed_probe.json 2> gpurun_out/seed_probe.err || { echo PROBE_FAILED; tail -30 gpurun_out/seed_probe.err; exit 1; }
cat gpurun_out/seed_probe.json
