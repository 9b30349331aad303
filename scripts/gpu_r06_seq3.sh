#!/bin/bash
# Round 6: third bisection of the first-step fault (scripts/diag/diag_first_step_seq.py, 8 ranks
# on one device over gloo; first the same staging order in one process, no gloo): libhgd's hop 1 with kernel arguments in host memory
# (HIP_FORCE_DEV_KERNARG=0), with copies on blit kernels instead of SDMA (HSA_ENABLE_SDMA=0),
# with the current stream drained before each all_reduce; a memory-bound torch gather as hop 1.
# Then the default bench line at HEAD. Records under gpurun_out/r06_seq/<tag>.
#   gpurun --timeout 1100 -- 'bash scripts/gpu_r06_seq3.sh <tag>'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06_seq/${1:-d}
mkdir -p $O
export TMPDIR=/tmp
( while sleep 45; do echo "[r06 seq3] $(date +%T) $(ls -t $O | head -1)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
run() {  # name, extra args
  timeout -k 10 150 python -u scripts/diag/diag_first_step_seq.py --world 8 --cycles 12 "${@:2}" \
      > $O/$1.jsonl 2> $O/$1.err && tail -1 $O/$1.jsonl
}
timeout -k 10 200 python -u scripts/diag/diag_stream_order.py --mode chunks --producer hgd,gather \
    --consumers d2h,d2d --trials 100 > $O/chunks_single.jsonl 2> $O/chunks_single.err && \
tail -1 $O/chunks_single.jsonl && \
run gather_torch --hop1 gather --hop2 torch && \
HIP_FORCE_DEV_KERNARG=0 run hgd_hgd_hostkernarg --hop1 hgd --hop2 hgd && \
HSA_ENABLE_SDMA=0 run hgd_hgd_nosdma --hop1 hgd --hop2 hgd && \
run hgd_hgd_sync --hop1 hgd --hop2 hgd --sync && \
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err && echo "bench ok" && \
cat $O/bench.json
rc=$?
echo "rc=$rc"
exit $rc
