#!/bin/bash
# Round 6: the blocked hop into items at other widths — A/B at d = 32 (P = 2, 3, 4) and the
# bench line (parity gate included) at d = 32 and d = 128. Records under gpurun_out/r06_dims/<tag>.
#   gpurun --timeout 1100 -- 'bash scripts/gpu_r06_dims.sh <tag>'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06_dims/${1:-a}
mkdir -p $O
export TMPDIR=/tmp
( while sleep 45; do echo "[r06 dims] $(date +%T) $(ls -t $O | head -1)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 200 python -u scripts/bench_mall_blocked.py --dim 32 --blocks 2,3,4 \
    > $O/ab_d32.json 2> $O/ab_d32.err && cat $O/ab_d32.json && \
timeout -k 10 400 python -u bench.py --dim 32 --pmc off > $O/bench_d32.json 2> $O/bench_d32.err && \
cat $O/bench_d32.json && \
timeout -k 10 500 python -u bench.py --dim 128 --pmc off > $O/bench_d128.json 2> $O/bench_d128.err && \
cat $O/bench_d128.json
rc=$?
echo "rc=$rc"
exit $rc
