#!/bin/bash
# Round 6: the source-blocked hop for the hop INTO USERS (gathers the 256 MB item table at
# d = 64, which the 256 MB Infinity Cache only partly holds next to the streams): plain vs
# P = 2, 3, 4 item ranges (scripts/bench_mall_blocked.py --hop users). Records under
# gpurun_out/r06_users/<tag>.
#   gpurun --timeout 900 -- 'bash scripts/gpu_r06_users.sh <tag>'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06_users/${1:-a}
mkdir -p $O
export TMPDIR=/tmp
( while sleep 45; do echo "[r06 users] $(date +%T) $(ls -t $O | head -1)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python -u scripts/bench_mall_blocked.py --hop users --dim 64 --blocks 2,3,4 \
    > $O/d64.json 2> $O/d64.err && cat $O/d64.json && \
timeout -k 10 300 python -u scripts/bench_mall_blocked.py --hop users --dim 128 --blocks 2,4,8 \
    --rounds 3 > $O/d128.json 2> $O/d128.err && cat $O/d128.json
rc=$?
echo "rc=$rc"
exit $rc
