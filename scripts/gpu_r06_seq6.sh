#!/bin/bash
# Round 6: sixth bisection — the staging round trip in 8 processes at once (no collective at all)
# with libhgd's hop, a torch matmul writer of the hop's duration, or a torch gather as the
# producer, and what the wrong rows hold (scripts/diag/diag_stream_order.py --mode chunks
# --roundtrip). Records under gpurun_out/r06_seq/<tag>.
#   gpurun --timeout 900 -- 'bash scripts/gpu_r06_seq6.sh <tag>'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06_seq/${1:-g}
mkdir -p $O
export TMPDIR=/tmp
( while sleep 45; do echo "[r06 seq6] $(date +%T) $(ls -t $O | head -1)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python -u scripts/diag/diag_stream_order.py --mode chunks --roundtrip \
    --producer hgd,mm,gather --rt-consumers clone --trials 25 --procs 8 \
    > $O/roundtrip_8procs.jsonl 2> $O/roundtrip_8procs.err && \
grep -v '"mode"' $O/roundtrip_8procs.jsonl | cut -c1-300
rc=$?
echo "rc=$rc"
exit $rc
