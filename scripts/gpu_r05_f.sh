#!/bin/bash
# Round 5: the Zipf over-bound steps 209/210 with hop-level checks of the compacted children.
#   gpurun --timeout 900 -- 'bash scripts/gpu_r05_f.sh <tag>'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/${1:-f}
mkdir -p $O
export TMPDIR=/tmp
( while sleep 45; do echo "[r05 f] $(date +%T) $(ls -t $O | head -1)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python -u scripts/diag/diag_zipf_teacher_forced.py --start 205 --stop 211 \
    --analyze 2 > $O/zipf_tf.jsonl 2> $O/zipf_tf.err
rc=$?
echo "zipf rc=$rc"; grep -c analysis $O/zipf_tf.jsonl; tail -c 300 $O/zipf_tf.jsonl
exit $rc
