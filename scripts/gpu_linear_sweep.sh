#!/bin/bash
# Row-GEMM / split-K microbench on one MI355X (scripts/bench_linear.py) over the workgroup caps in
# $BLOCKS (default 512), rows 69,716 / 31,668 at d = 64 and 144,242 at d = 128.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/lin
for b in ${BLOCKS:-512}; do
  HGD_ROWGEMM_BLOCKS=$b timeout -k 10 120 python scripts/bench_linear.py --rows 69716 31668 > gpurun_out/lin/b$b.jsonl 2>&1 || { cat gpurun_out/lin/b$b.jsonl; exit 1; }
  HGD_ROWGEMM_BLOCKS=$b timeout -k 10 120 python scripts/bench_linear.py --rows 144242 --dim 128 >> gpurun_out/lin/b$b.jsonl 2>&1 || { cat gpurun_out/lin/b$b.jsonl; exit 1; }
done
grep -h hgd gpurun_out/lin/*.jsonl
