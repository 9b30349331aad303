#!/bin/bash
# Round 6: cache policy of the blocked hop into items at d = 64 — does keeping the index / weight
# streams and the Y partials out of the caches (non-temporal) leave more of the Infinity Cache to
# the gathered user slice? Policies 8 (default), 9 (+ nt Y stores), 10 (+ nt index loads), 11
# (all), plain and P = 4, 5, 8 each (scripts/bench_mall_blocked.py --policy).
# Records under gpurun_out/r06_policy/<tag>.
#   gpurun --timeout 900 -- 'bash scripts/gpu_r06_policy.sh <tag>'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06_policy/${1:-a}
mkdir -p $O
export TMPDIR=/tmp
( while sleep 45; do echo "[r06 policy] $(date +%T) $(ls -t $O | head -1)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for pol in 8 9 10 11; do
  timeout -k 10 200 python -u scripts/bench_mall_blocked.py --dim 64 --blocks 4,5,8 \
      --policy $pol > $O/pol$pol.json 2> $O/pol$pol.err || exit 1
  cat $O/pol$pol.json
done
echo "rc=0"
