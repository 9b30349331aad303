#!/bin/bash
# Round 6: the blocked hop into items with each block's short rows walked by the segmented
# kernel (HGD_TUNE_SPMM_BLOCKED_SEG = 1) vs a lane group per row (0): its bitwise test, then
# d = 64 at P = 4, 5, 8, 10 and d = 128 at P = 8, 12, 16 (scripts/bench_mall_blocked.py --seg).
# Records under gpurun_out/r06_bseg/<tag>.
#   gpurun --timeout 900 -- 'bash scripts/gpu_r06_bseg.sh <tag>'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06_bseg/${1:-a}
mkdir -p $O
export TMPDIR=/tmp
( while sleep 45; do echo "[r06 bseg] $(date +%T) $(ls -t $O | head -1)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_spmm.py -k "block" > $O/pytest.txt 2>&1 && tail -1 $O/pytest.txt || exit 1
for seg in 0 1; do
  timeout -k 10 200 python -u scripts/bench_mall_blocked.py --dim 64 --blocks 4,5,8,10 \
      --seg $seg > $O/d64_seg$seg.json 2> $O/d64_seg$seg.err || exit 1
  cat $O/d64_seg$seg.json
  timeout -k 10 250 python -u scripts/bench_mall_blocked.py --dim 128 --blocks 8,12,16 \
      --seg $seg --rounds 3 > $O/d128_seg$seg.json 2> $O/d128_seg$seg.err || exit 1
  cat $O/d128_seg$seg.json
done
echo "rc=0"
