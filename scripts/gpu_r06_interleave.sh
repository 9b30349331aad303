#!/bin/bash
# Round 6: HGD_TUNE_SPMM_PASS_INTERLEAVE (a wide row's column passes as one XCD-interleaved
# launch): its bitwise GPU test, the hop A/B at the bench graph for d = 256 (and 192, 512), then
# bench.py --dim 256 with it on (the parity gate included) for the line's own number.
# Records under gpurun_out/r06_interleave/<tag>.
#   gpurun --timeout 1200 -- 'bash scripts/gpu_r06_interleave.sh <tag>'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06_interleave/${1:-a}
mkdir -p $O
export TMPDIR=/tmp
( while sleep 45; do echo "[r06 interleave] $(date +%T) $(ls -t $O | head -1)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    -m gpu tests/test_gpu_spmm.py > $O/pytest_spmm.txt 2>&1 && tail -1 $O/pytest_spmm.txt && \
timeout -k 10 300 python -u scripts/bench_pass_interleave.py --dim 256 > $O/ab_d256.json \
    2> $O/ab_d256.err && cat $O/ab_d256.json && \
timeout -k 10 300 python -u scripts/bench_pass_interleave.py --dim 512 --edges 50000000 \
    > $O/ab_d512.json 2> $O/ab_d512.err && cat $O/ab_d512.json && \
HGD_SPMM_PASS_INTERLEAVE=1 timeout -k 10 900 python -u bench.py --dim 256 \
    > $O/bench_d256_interleave.json 2> $O/bench_d256_interleave.err && echo "bench ok" && \
tail -c 1500 $O/bench_d256_interleave.json
rc=$?
echo "rc=$rc"
exit $rc
