#!/bin/bash
# Round 6: fourth bisection of the first-step fault. (1) the single-process staging test of
# diag_stream_order.py --mode chunks run by 8 processes at once on the device (contention, no
# gloo); (2) the 8-rank sequence with gloo's staging restated in torch calls (--reduce emul),
# without and with the current stream drained first; (3) libhgd's hop with the real gloo
# all-reduce and the stream drained (the library's fix). Records under gpurun_out/r06_seq/<tag>.
#   gpurun --timeout 1100 -- 'bash scripts/gpu_r06_seq4.sh <tag>'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06_seq/${1:-e}
mkdir -p $O
export TMPDIR=/tmp
( while sleep 45; do echo "[r06 seq4] $(date +%T) $(ls -t $O | head -1)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
python -c "import torch; print('current stream', torch.cuda.current_stream().cuda_stream, torch._C._cuda_getCurrentRawStream(0))" > $O/streams.txt 2>&1
cat $O/streams.txt
run() {  # name, extra args
  timeout -k 10 150 python -u scripts/diag/diag_first_step_seq.py --world 8 --cycles 12 "${@:2}" \
      > $O/$1.jsonl 2> $O/$1.err && tail -1 $O/$1.jsonl
}
timeout -k 10 240 python -u scripts/diag/diag_stream_order.py --mode chunks --producer hgd \
    --consumers d2h --trials 60 --procs 8 > $O/chunks_8procs.jsonl 2> $O/chunks_8procs.err && \
grep '"mode"' $O/chunks_8procs.jsonl | cut -c1-220 && \
run hgd_hgd_emul --hop1 hgd --hop2 hgd --reduce emul && \
run hgd_hgd_emul_sync --hop1 hgd --hop2 hgd --reduce emul --sync && \
run hgd_hgd_sync --hop1 hgd --hop2 hgd --sync
rc=$?
echo "rc=$rc"
exit $rc
