#!/bin/bash
# Round 6: cache policy of the hop into users at d = 64 (plain hop; the item table is the
# Infinity-Cache candidate): policies 8 (default), 9, 10, 11 (scripts/bench_mall_blocked.py
# --hop users --blocks 1, i.e. the plain hop only). Records under gpurun_out/r06_policy/<tag>.
#   gpurun --timeout 900 -- 'bash scripts/gpu_r06_policy_users.sh <tag>'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06_policy/${1:-users}
mkdir -p $O
export TMPDIR=/tmp
( while sleep 45; do echo "[r06 policy] $(date +%T) $(ls -t $O | head -1)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for pol in 8 9 10 11 1 0; do
  timeout -k 10 200 python -u scripts/bench_mall_blocked.py --hop users --dim 64 --blocks 1 \
      --policy $pol > $O/users_pol$pol.json 2> $O/users_pol$pol.err || exit 1
  cat $O/users_pol$pol.json
done
echo "rc=0"
