#!/bin/bash
# B = 64 / 128 / 256: the shipped plan vs the register-resident kernel forced (flag 1 << 23) with
# 256 splits (shipped build: pre-pass seeded) and with 128 (AHR_QRES_SMALLB_SPLITS=128: self-seeded)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/qs128}; mkdir -p $O
L=ah-rag_amd/ah_rag/_lib
for r in 1 2; do
  for v in libahr_hip.so variant_qs128/libahr_hip.so; do
    n=$(echo $v | tr '/' '_')
    AHR_LIB_PATH=$L/$v timeout -k 10 300 python -u tools/dense_ablation.py --workload hotpot90k --batches 64,128,256 --variants prod:-1:0,qres:-1:8388608 --rounds 2 --steps 40 > $O/${n}_r$r.json 2> $O/${n}_r$r.err || { echo FAIL $v; tail -5 $O/${n}_r$r.err; exit 1; }
    python - $O/${n}_r$r.json $n <<'PY'
import json, sys
for line in open(sys.argv[1]):
    d = json.loads(line)
    print(sys.argv[2], d["B"], {k: (d[k]["tile_topk"], round(sum(d[k].values()), 4)) for k in ("prod", "qres")})
PY
  done
done
