#!/bin/bash
# Round 5, third GPU pass (records under gpurun_out/r05/<tag>):
#   gpurun --timeout 1200 -- 'bash scripts/gpu_r05_c.sh <tag>'
#   1. masked-walk bitwise tests (push permutes), the LastFM seed sweep at 1e-5 outright, the
#      plugin suite with graph replay as the HCCF default, the graph-step tests;
#   2. the masked hop micro-bench (push / pull / one-batch) and the HCCF step variants;
#   3. the Zipf teacher-forced record with the first over-bound steps decomposed.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/${1:-c}
mkdir -p $O
export TMPDIR=/tmp
( while sleep 45; do echo "[r05 c] $(date +%T) $(ls -t $O | head -1)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 900 python -u -m pytest tests/test_gpu_masked_pair.py tests/test_gpu_plugins.py \
    tests/test_gpu_graph_step.py "tests/test_gpu_config_parity.py::test_hccf_lastfm_seeds_row_bound" \
    -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.txt 2>&1
prc=$?
grep -E "passed|failed" $O/pytest.txt | tail -2
[ $prc -eq 0 ] || [ $prc -eq 1 ] || exit $prc
timeout -k 10 300 python -u scripts/bench_masked_hop.py > $O/masked_hop.json 2> $O/masked_hop.err && \
cat $O/masked_hop.json && \
timeout -k 10 300 python -u scripts/bench_hccf.py --reps 30 \
    --variants hgd_cs_eager_cpu_mask,hgd_graph_ref_adam,hgd_graph_cpu_mask > $O/hccf.jsonl 2> $O/hccf.err && \
cat $O/hccf.jsonl && \
timeout -k 10 700 python -u scripts/diag/diag_zipf_teacher_forced.py --start 200 --stop 250 \
    --analyze 4 > $O/zipf_tf.jsonl 2> $O/zipf_tf.err
rc=$?
echo "rc=$rc"; grep -c analysis $O/zipf_tf.jsonl
exit $(( rc ? rc : prc ))
