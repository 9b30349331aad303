#!/bin/bash
# Round 2 re-entry check: whole GPU suite, smoke, N=1 headline bench, HCCF step bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_c.log 2>&1 || { tail -30 gpurun_out/pytest_c.log; exit 1; }
tail -3 gpurun_out/pytest_c.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_c.log 2>&1 || { tail -20 gpurun_out/smoke_c.log; exit 1; }
cat gpurun_out/smoke_c.log
timeout -k 10 300 python bench.py > gpurun_out/bench_c.json 2> gpurun_out/bench_c.err || { tail -20 gpurun_out/bench_c.err; exit 1; }
cat gpurun_out/bench_c.json
timeout -k 10 300 python scripts/bench_hccf.py > gpurun_out/hccf_c.log 2>&1 || { tail -20 gpurun_out/hccf_c.log; exit 1; }
tail -8 gpurun_out/hccf_c.log
echo ALL_OK
