#!/bin/bash
# Round 2, first GPU pass: GPU tests, the 2-rank strong-scaling rehearsal (gloo on one device),
# the N=1 headline bench, d=256 and the sliced-hop cost at N=1.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_a.log 2>&1 || { tail -30 gpurun_out/pytest_a.log; exit 1; }
tail -3 gpurun_out/pytest_a.log
HGD_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 1 --check \
  --no-cpu-baseline > gpurun_out/bench_g2_check.json 2> gpurun_out/bench_g2_check.err || { tail -20 gpurun_out/bench_g2_check.err; exit 1; }
cat gpurun_out/bench_g2_check.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err || { tail -20 gpurun_out/bench_n1.err; exit 1; }
cat gpurun_out/bench_n1.json
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --slice-width 32 --no-cpu-baseline --pmc off > gpurun_out/bench_n1_sliced.json 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --dim 256 --no-cpu-baseline --pmc off > gpurun_out/bench_n1_d256.json 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --dim 256 --slice-width 64 --no-cpu-baseline --pmc off > gpurun_out/bench_n1_d256_sliced.json 2>&1 || exit 1
echo ALL_OK
