#!/bin/bash
# Round 5: the committed Zipf record — epoch 2 batches 150.. end teacher-forced against float64
# (exact dropout masks), no decomposition. gpurun --timeout 1200 -- 'bash scripts/gpu_r05_g.sh <tag>'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/${1:-g}
mkdir -p $O
export TMPDIR=/tmp
( while sleep 45; do echo "[r05 g] $(date +%T) $(tail -c 120 $O/zipf_tf.jsonl 2>/dev/null)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 1100 python -u scripts/diag/diag_zipf_teacher_forced.py --start ${START:-150} \
    --stop 10000 --analyze 0 > $O/zipf_tf.jsonl 2> $O/zipf_tf.err
rc=$?
echo "zipf rc=$rc"; tail -c 300 $O/zipf_tf.jsonl
exit $rc
