#!/bin/bash
# Whole GPU suite, HCCF step bench, ED-HNN block bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/d
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/d/pytest.log 2>&1 || { tail -30 gpurun_out/d/pytest.log; exit 1; }
tail -2 gpurun_out/d/pytest.log
timeout -k 10 300 python scripts/bench_hccf.py > gpurun_out/d/hccf.jsonl 2>&1 || { tail -20 gpurun_out/d/hccf.jsonl; exit 1; }
grep variant gpurun_out/d/hccf.jsonl
timeout -k 10 300 python scripts/bench_edhnn.py > gpurun_out/d/edhnn.jsonl 2>&1 || { tail -20 gpurun_out/d/edhnn.jsonl; exit 1; }
tail -6 gpurun_out/d/edhnn.jsonl
