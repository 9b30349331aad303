#!/bin/bash
# Round 6: the ordering of gloo's staging copy behind the kernel that produced its input
# (scripts/diag/diag_stream_order.py), on one MI355X. Records under gpurun_out/r06_order/<tag>.
#   gpurun --timeout 900 -- 'bash scripts/gpu_r06_order.sh <tag>'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06_order/${1:-a}
mkdir -p $O
export TMPDIR=/tmp
( while sleep 45; do echo "[r06 order] $(date +%T) $(ls -t $O | head -1)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python -u scripts/diag/diag_stream_order.py --mode single --trials 200 \
    > $O/single.jsonl 2> $O/single.err && echo "single ok" && \
HSA_ENABLE_SDMA=0 timeout -k 10 300 python -u scripts/diag/diag_stream_order.py --mode single \
    --trials 200 --consumers d2h,d2d > $O/single_nosdma.jsonl 2> $O/single_nosdma.err && \
echo "single nosdma ok" && \
timeout -k 10 400 python -u scripts/diag/diag_stream_order.py --mode gloo --world 8 --cycles 40 \
    > $O/gloo8.jsonl 2> $O/gloo8.err && echo "gloo ok" && \
HSA_ENABLE_SDMA=0 timeout -k 10 400 python -u scripts/diag/diag_stream_order.py --mode gloo \
    --world 8 --cycles 40 > $O/gloo8_nosdma.jsonl 2> $O/gloo8_nosdma.err && echo "gloo nosdma ok"
rc=$?
echo "rc=$rc"
exit $rc
