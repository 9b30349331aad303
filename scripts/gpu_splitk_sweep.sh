#!/bin/bash
# Split-K rows-per-slice sweep (HGD_SPLITK_ROWS) of the weight-gradient product at the carriers'
# shapes: rows 69,716 / 31,668 at d = 64, 144,242 at d = 128 (scripts/bench_linear.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/splitk
mkdir -p $O
for r in auto 64 128 192 256 384 512 1024; do
  if [ $r = auto ]; then unset HGD_SPLITK_ROWS; else export HGD_SPLITK_ROWS=$r; fi
  timeout -k 10 120 python scripts/bench_linear.py --rows 69716 31668 > $O/r$r.jsonl 2>&1 || { cat $O/r$r.jsonl; exit 1; }
  timeout -k 10 120 python scripts/bench_linear.py --rows 144242 --dim 128 >> $O/r$r.jsonl 2>&1 || { cat $O/r$r.jsonl; exit 1; }
done
grep -h bwd_weight_hgd $O/*.jsonl
