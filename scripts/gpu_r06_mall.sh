#!/bin/bash
# Round 6: the source-blocked hop into items (hgd_spmm_blocked): its GPU tests, then the A/B
# against hgd_spmm at the bench graph for d = 64, 128, 256 (scripts/bench_mall_blocked.py), then
# the default bench line. Records under gpurun_out/r06_mall/<tag>.
#   gpurun --timeout 1100 -- 'bash scripts/gpu_r06_mall.sh <tag>'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06_mall/${1:-b}
mkdir -p $O
export TMPDIR=/tmp
( while sleep 45; do echo "[r06 mall] $(date +%T) $(ls -t $O | head -1)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_spmm.py -k "block" > $O/pytest_blocked.log 2>&1 && tail -3 $O/pytest_blocked.log && \
timeout -k 10 300 python -u scripts/bench_mall_blocked.py --dim 64 --blocks 3,4,5,6 \
    > $O/d64.json 2> $O/d64.err && cat $O/d64.json && \
timeout -k 10 300 python -u scripts/bench_mall_blocked.py --dim 128 --blocks 6,8,10 \
    > $O/d128.json 2> $O/d128.err && cat $O/d128.json && \
timeout -k 10 400 python -u scripts/bench_mall_blocked.py --dim 256 --blocks 3,4,5,6 \
    --rounds 3 > $O/d256.json 2> $O/d256.err && cat $O/d256.json && \
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err && cat $O/bench.json
rc=$?
echo "rc=$rc"
exit $rc
