#!/bin/bash
# Round 6: fifth bisection of the first-step fault — gloo's whole staging cycle (D2H, host op,
# H2D back, a consumer kernel) in one process and in 8 processes at once, libhgd's hop or a torch
# gather as the producer (scripts/diag/diag_stream_order.py --mode chunks --roundtrip); then the
# default bench line at HEAD. Records under gpurun_out/r06_seq/<tag>.
#   gpurun --timeout 1100 -- 'bash scripts/gpu_r06_seq5.sh <tag>'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06_seq/${1:-f}
mkdir -p $O
export TMPDIR=/tmp
( while sleep 45; do echo "[r06 seq5] $(date +%T) $(ls -t $O | head -1)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 240 python -u scripts/diag/diag_stream_order.py --mode chunks --roundtrip \
    --producer hgd,gather --trials 60 > $O/roundtrip_1proc.jsonl 2> $O/roundtrip_1proc.err && \
grep -v '"mode"' $O/roundtrip_1proc.jsonl && \
timeout -k 10 300 python -u scripts/diag/diag_stream_order.py --mode chunks --roundtrip \
    --producer hgd,gather --trials 30 --procs 8 > $O/roundtrip_8procs.jsonl \
    2> $O/roundtrip_8procs.err && grep -v '"mode"' $O/roundtrip_8procs.jsonl | grep "proc 0\]" && \
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err && echo "bench ok" && \
cat $O/bench.json
rc=$?
echo "rc=$rc"
exit $rc
