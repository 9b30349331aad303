#!/bin/bash
# Round 5, second GPU pass (records under gpurun_out/r05/<tag>):
#   gpurun --timeout 1200 -- 'bash scripts/gpu_r05_b.sh <tag>'
#   1. InfoNCE / config-parity / graph-step / HCCF plugin / p2p tests after the accurate-diagonal
#      InfoNCE change and the P2PExchange lifetime change;
#   2. the per-seed ratio table (ours vs the reference's own fp32);
#   3. the Zipf two-epoch divergence, teacher-forced against float64 from epoch 2 batch 200 on;
#   4. Adam variants against the reference's Adam, bit for bit over 50 HCCF steps, and the HCCF
#      step variants (eager default, graph replays, graph with the reference's Adam after it).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/${1:-b}
mkdir -p $O
export TMPDIR=/tmp
( while sleep 45; do echo "[r05 b] $(date +%T) $(ls -t $O | head -1)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 900 python -u -m pytest tests/test_gpu_infonce.py tests/test_gpu_config_parity.py \
    tests/test_gpu_graph_step.py tests/test_gpu_plugins.py tests/test_gpu_p2p.py -v \
    --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.txt 2>&1
prc=$?
tail -3 $O/pytest.txt
[ $prc -eq 0 ] || [ $prc -eq 1 ] || exit $prc   # 1 = test failures: still run the diagnostics
timeout -k 10 300 python -u scripts/diag/diag_view_ratio.py > $O/seed_ratios.jsonl 2> $O/seed_ratios.err && \
echo "ratios ok" && \
timeout -k 10 900 python -u scripts/diag/diag_zipf_teacher_forced.py --start 200 > $O/zipf_tf.jsonl 2> $O/zipf_tf.err
rc=$?
echo "diag rc=$rc"; tail -c 600 $O/zipf_tf.jsonl
[ $rc -eq 0 ] && timeout -k 10 300 python -u scripts/diag/diag_adam_bitwise.py > $O/adam_bitwise.jsonl 2> $O/adam_bitwise.err && \
cat $O/adam_bitwise.jsonl && \
timeout -k 10 300 python -u scripts/bench_hccf.py --reps 30 \
    --variants hgd_cs_eager_cpu_mask,hgd_graph_cpu_mask,hgd_graph_ref_adam,hgd_graph > $O/hccf.jsonl 2> $O/hccf.err && \
cat $O/hccf.jsonl
rc=$?
exit $(( rc ? rc : prc ))
