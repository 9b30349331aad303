#!/bin/bash
# Round 6: (1) scripts/diag/diag_p2p_first.py once, as VERDICT r05 asked, without
# --sync-before-allreduce — the library's sharded ops now drain the producing stream before every
# gloo collective themselves (sharded.ordered_all_reduce); (2) the 8-process staging round trip
# with each Ms block snapshotted before its producer (what the wrong rows held).
# Records under gpurun_out/r06_seq/<tag>.
#   gpurun --timeout 1100 -- 'bash scripts/gpu_r06_seq8.sh <tag>'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06_seq/${1:-i}
mkdir -p $O
export TMPDIR=/tmp
( while sleep 45; do echo "[r06 seq8] $(date +%T) $(ls -t $O | head -1)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 420 python -u scripts/diag/diag_p2p_first.py --world 8 --cycles 12 \
    > $O/p2p_first_n8.jsonl 2> $O/p2p_first_n8.err && tail -1 $O/p2p_first_n8.jsonl && \
bash scripts/gpu_r06_seq7.sh ${1:-i}
rc=$?
echo "rc=$rc"
exit $rc
