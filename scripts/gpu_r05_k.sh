#!/bin/bash
# Round 5: optim.ReferenceAdam (the reference's Adam as one capturable kernel): its tests, the
# plugin graph tests, the Adam bitwise diag, the HCCF step variants; then the N = 2 / 8
# default-flag bench rehearsals. gpurun --timeout 1200 -- 'bash scripts/gpu_r05_k.sh <tag>'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/${1:-k}
mkdir -p $O
export TMPDIR=/tmp
( while sleep 45; do echo "[r05 k] $(date +%T) $(ls -t $O | head -1)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 120 python -u scripts/diag/diag_adam_ops.py > $O/adam_ops.json 2> $O/adam_ops.err && \
cat $O/adam_ops.json && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_adam.py tests/test_gpu_graph_step.py \
    tests/test_gpu_plugins.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/pytest.txt 2>&1 && tail -1 $O/pytest.txt && \
timeout -k 10 300 python -u scripts/diag/diag_adam_bitwise.py > $O/adam_bitwise.jsonl 2> $O/adam_bitwise.err && \
cat $O/adam_bitwise.jsonl && \
timeout -k 10 300 python -u scripts/bench_hccf.py --reps 50 \
    --variants hgd_graph_kernel_adam,hgd_graph_ref_adam,hgd_graph_cpu_mask,hgd_cs_eager_cpu_mask > $O/hccf.jsonl 2> $O/hccf.err && \
cat $O/hccf.jsonl || exit 1
kill $HB 2>/dev/null
REH_N="2 8" bash scripts/gpu_r05_d.sh ${1:-k}
