#!/bin/bash
# Round 6: second bisection of the first-step fault (scripts/diag/diag_first_step_seq.py):
# libhgd's producer followed by a tiny torch kernel, one item chunk per slice, 4 ranks, libhgd's producer
# with the current stream drained before each all_reduce; then the default bench line at HEAD.
# Records under gpurun_out/r06_seq/<tag>.
#   gpurun --timeout 1100 -- 'bash scripts/gpu_r06_seq2.sh <tag>'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06_seq/${1:-b}
mkdir -p $O
export TMPDIR=/tmp
( while sleep 45; do echo "[r06 seq2] $(date +%T) $(ls -t $O | head -1)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
run() {  # name, extra args
  timeout -k 10 240 python -u scripts/diag/diag_first_step_seq.py --world 8 --cycles 12 "${@:2}" \
      > $O/$1.jsonl 2> $O/$1.err && tail -1 $O/$1.jsonl
}
run hgd_torch_tail --hop1 hgd --hop2 torch --tail && \
run hgd_hgd_chunks1 --hop1 hgd --hop2 hgd --chunks 1 && \
run hgd_hgd_world4 --hop1 hgd --hop2 hgd --world 4 && \
run hgd_hgd_sync --hop1 hgd --hop2 hgd --sync && \
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err && echo "bench ok" && \
cat $O/bench.json
rc=$?
echo "rc=$rc"
exit $rc
