#!/bin/bash
# Cost of the column-slice pipeline's narrower hops at N=1 (no exchange): d=64 in slices of
# 64/32/16 columns, d=256 in slices of 256/128/64/32.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/slices
export TMPDIR=/tmp
for w in 64 32 16; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --slice-width $w --no-cpu-baseline --pmc off \
    > gpurun_out/slices/d64_w$w.json 2> gpurun_out/slices/d64_w$w.err || exit 1
done
for w in 128 64 32; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --dim 256 --slice-width $w --no-cpu-baseline --pmc off \
    > gpurun_out/slices/d256_w$w.json 2> gpurun_out/slices/d256_w$w.err || exit 1
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/slices/*.json")):
    j = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, j["value"], j["ms_per_step"], j["roofline"]["frac"])
PY
