#!/bin/bash
# Same-box A/B of library builds on the small-batch kernels (tools/small_ab.py: bf16 B = 1, 4 and
# fp32 B = 1, 4 on the C2 corpus; warm / cold), after the fp32 and small-kernel parity tests on the
# in-tree build. usage: bash tools/gpu/small_libs.sh OUT ROUNDS LIB...   (labels: directory names)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$1; R=$2; shift 2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_dense_gpu.py tests/test_configs_gpu.py -m gpu -x -q -k "f32 or small" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in $(seq 1 $R); do for lib in "$@"; do
  v=$(basename $(dirname $lib))
  AHR_LIB_PATH=$lib timeout -k 10 300 python -u tools/small_ab.py --batches 1,4 --reps 100 > $O/ab_${v}_r$r.json 2> $O/ab_${v}_r$r.err || { echo AB_FAIL; tail -5 $O/ab_${v}_r$r.err; exit 1; }
  python -c "
import json,sys; d=json.load(open(sys.argv[1]))
print(sys.argv[2], *[(b, d[b]['warm_us'].get('tile_topk'), d[b]['cold_us'].get('tile_topk'), 'sum', round(sum(d[b]['warm_us'].values()), 2)) for b in ('f32_b1','f32_b4','bf16_b1','bf16_b4')])" $O/ab_${v}_r$r.json $v
done; done
