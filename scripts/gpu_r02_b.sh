#!/bin/bash
# Round 2: config-shape parity tests + the d=128/256 column-pass A/B of the hop.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_config_parity.py -x -v -s --timeout 400 \
  --timeout-method thread > gpurun_out/pytest_cfg.log 2>&1 || { tail -60 gpurun_out/pytest_cfg.log; exit 1; }
grep -E "worst row|PASS|FAIL" gpurun_out/pytest_cfg.log
for pc in 256 128 64; do
  HGD_SPMM_PASS_COLS=$pc timeout -k 10 300 python bench.py --steps 10 --warmup 3 --dim 256 --no-cpu-baseline --pmc off > gpurun_out/bench_d256_pc$pc.json 2>&1 || exit 1
  HGD_SPMM_PASS_COLS=$pc timeout -k 10 300 python bench.py --steps 10 --warmup 3 --dim 128 --no-cpu-baseline --pmc off > gpurun_out/bench_d128_pc$pc.json 2>&1 || exit 1
done
echo ALL_OK
