#!/bin/bash
# Round 5, first GPU pass (records under gpurun_out/r05/<tag>):
#   gpurun --timeout 1200 -- 'bash scripts/gpu_r05_a.sh <tag>'
#   1. the LastFM seed sweep (seeds 10-19, compacted + view) and the x3p queue-form test;
#   2. the per-seed ratio table (ours vs the reference's own fp32, scripts/diag/diag_view_ratio.py);
#   3. the default bench line with its same-run parity gate.
# Each step has its own limit; the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/${1:-a}
mkdir -p $O
export TMPDIR=/tmp
( while sleep 45; do echo "[r05 a] $(date +%T) $(ls -t $O | head -1)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_config_parity.py tests/test_gpu_linear.py \
    -k "lastfm_seeds or x3p_queue or masked_drop_views" -v -s --timeout 300 \
    --timeout-method thread -p no:cacheprovider > $O/pytest.txt 2>&1
prc=$?
tail -3 $O/pytest.txt
[ $prc -eq 0 ] || [ $prc -eq 1 ] || exit $prc   # 1 = test failures: still run the table
timeout -k 10 300 python -u scripts/diag/diag_view_ratio.py > $O/seed_ratios.jsonl 2> $O/seed_ratios.err && \
echo "ratios ok" && \
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?
echo "bench rc=$rc"; tail -c 1500 $O/bench.json
exit $(( rc ? rc : prc ))
