#!/bin/bash
# Round 6: can the d = 256 hop into items (configs[4]'s width) use the source-blocked hop with
# wider column passes? Default 64-column passes vs 128- and 256-column passes, each plain and
# blocked (scripts/bench_mall_blocked.py). Records under gpurun_out/r06_wide/<tag>.
#   gpurun --timeout 900 -- 'bash scripts/gpu_r06_wide.sh <tag>'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06_wide/${1:-a}
mkdir -p $O
export TMPDIR=/tmp
( while sleep 45; do echo "[r06 wide] $(date +%T) $(ls -t $O | head -1)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python -u scripts/bench_mall_blocked.py --dim 256 --pass-cols 128 \
    --blocks 4,8,12 --rounds 3 > $O/p128.json 2> $O/p128.err && cat $O/p128.json && \
timeout -k 10 300 python -u scripts/bench_mall_blocked.py --dim 256 --pass-cols 256 \
    --blocks 8,16 --rounds 3 > $O/p256.json 2> $O/p256.err && cat $O/p256.json
rc=$?
echo "rc=$rc"
exit $rc
