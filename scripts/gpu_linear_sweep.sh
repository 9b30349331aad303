#!/bin/bash
# A/B of the skinny-product kernel variants at the carriers' shapes (one process per setting;
# HGD_GEMM_EXACT=1 is the f32-MFMA baseline, HGD_X3_COLS the split-bf16 row GEMM's slice width,
# HGD_X3_SPLITK the split-K form). Records under gpurun_out/linsweep/.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/linsweep
mkdir -p $O
export TMPDIR=/tmp
if [ "${SWEEP_TESTS:-1}" = 1 ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_linear.py tests/test_gpu_fused_dropout.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
for cfg in ${SWEEP_CFGS:-"HGD_GEMM_EXACT=1" "HGD_X3_COLS=0" "HGD_X3_COLS=128" "HGD_X3_SPLITK=0"}; do
  tag=$(echo $cfg | tr '=' '_')
  env $cfg timeout -k 10 120 python scripts/bench_linear.py --rows 144242 --dim 128 > $O/d128_$tag.jsonl 2>&1 || { cat $O/d128_$tag.jsonl; exit 1; }
  env $cfg timeout -k 10 120 python scripts/bench_linear.py --rows 69716 31668 --dim 64 > $O/d64_$tag.jsonl 2>&1 || { cat $O/d64_$tag.jsonl; exit 1; }
  echo "== $cfg"
  python3 - $O/d128_$tag.jsonl $O/d64_$tag.jsonl <<'PY'
import json, sys
for f in sys.argv[1:]:
    for l in open(f):
        if l.startswith("{"):
            r = json.loads(l)
            if r["case"].endswith("_hgd"):
                print(f"  {r['case']:18s} rows {r['rows']:7d} d {r['d']:4d} {r['us']:8.2f} us {r['alg_GBps']:8.1f} GB/s")
PY
done
