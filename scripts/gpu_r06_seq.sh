#!/bin/bash
# Round 6: bisect the one-device gloo rehearsal's first-step fault with the exact two_hop call
# sequence (scripts/diag/diag_first_step_seq.py): torch hops, libhgd hops, and the mix.
# Records under gpurun_out/r06_seq/<tag>.
#   gpurun --timeout 1000 -- 'bash scripts/gpu_r06_seq.sh <tag>'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06_seq/${1:-a}
mkdir -p $O
export TMPDIR=/tmp
( while sleep 45; do echo "[r06 seq] $(date +%T) $(ls -t $O | head -1)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
run() {  # name, extra args
  timeout -k 10 300 python -u scripts/diag/diag_first_step_seq.py --world 8 --cycles 12 "${@:2}" \
      > $O/$1.jsonl 2> $O/$1.err && tail -1 $O/$1.jsonl
}
run torch_torch --hop1 torch --hop2 torch && \
run hgd_hgd --hop1 hgd --hop2 hgd && \
run hgd_torch --hop1 hgd --hop2 torch && \
run torch_hgd --hop1 torch --hop2 hgd
rc=$?
echo "rc=$rc"
exit $rc
