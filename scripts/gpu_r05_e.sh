#!/bin/bash
# Round 5: the Zipf over-bound steps 209/210 with hop-level checks of the compacted children,
# then the N = 4 default-flag bench rehearsal (scripts/gpu_r05_d.sh). Records under
# gpurun_out/r05/<tag>.   gpurun --timeout 1200 -- 'bash scripts/gpu_r05_e.sh <tag>'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/${1:-e}
mkdir -p $O
export TMPDIR=/tmp
( while sleep 45; do echo "[r05 e] $(date +%T) $(ls -t $O | head -1)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 500 python -u scripts/diag/diag_zipf_teacher_forced.py --start 205 --stop 211 \
    --analyze 2 > $O/zipf_tf.jsonl 2> $O/zipf_tf.err
rc=$?
echo "zipf rc=$rc"; grep -c analysis $O/zipf_tf.jsonl
[ $rc -eq 0 ] || exit $rc
kill $HB 2>/dev/null
bash scripts/gpu_r05_d.sh ${1:-e}
