set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in tl_gemm:34 kb_gemm:524290 kb256_gemm:131074; do
  name=${cfg%%:*}; fl=${cfg##*:}
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/fa_$name/fetch --output-format csv -- python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --inflight 1 --debug-flags $fl > gpurun_out/fa_$name.log 2>&1 || { echo FAIL $name; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d gpurun_out/fa_$name/ea --output-format csv -- python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --inflight 1 --debug-flags $fl > gpurun_out/fa_$name.log 2>&1 || { echo FAIL2 $name; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/fa_$name/l2 --output-format csv -- python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --inflight 1 --debug-flags $fl > gpurun_out/fa_$name.log 2>&1 || { echo FAIL3 $name; exit 1; }
  python tools/sq_summary.py gpurun_out/fa_$name > gpurun_out/fa_$name.json
  cat gpurun_out/fa_$name.json
done
