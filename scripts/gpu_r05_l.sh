#!/bin/bash
# Round 5: the step-table ReferenceAdam (vectorised kernel, device row index): Adam / graph /
# plugin tests, the Adam bitwise diag, the HCCF step variants and the plugin epoch.
#   gpurun --timeout 1200 -- 'bash scripts/gpu_r05_l.sh <tag>'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/${1:-l}
mkdir -p $O
export TMPDIR=/tmp
( while sleep 45; do echo "[r05 l] $(date +%T) $(ls -t $O | head -1)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_adam.py tests/test_gpu_graph_step.py \
    tests/test_gpu_plugins.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/pytest.txt 2>&1 && tail -1 $O/pytest.txt && \
timeout -k 10 300 python -u scripts/diag/diag_adam_bitwise.py > $O/adam_bitwise.jsonl 2> $O/adam_bitwise.err && \
tail -1 $O/adam_bitwise.jsonl && \
timeout -k 10 300 python -u scripts/bench_hccf.py --reps 50 \
    --variants hgd_graph_kernel_adam,hgd_graph_ref_adam,hgd_graph_cpu_mask,hgd_cs_eager_cpu_mask > $O/hccf.jsonl 2> $O/hccf.err && \
cat $O/hccf.jsonl && \
timeout -k 10 300 python -u scripts/bench_plugin_epoch.py > $O/plugin_epoch.json 2> $O/plugin_epoch.err && \
tail -c 600 $O/plugin_epoch.json
