#!/bin/bash
# Round 5: host-time profile of the replayed HCCF step, the graph / plugin tests after the slot
# consolidation, and the HCCF step variants. gpurun --timeout 900 -- 'bash scripts/gpu_r05_n.sh <tag>'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/${1:-n}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 python -u scripts/profile_graph_step_host.py > $O/host.json 2> $O/host.err && \
cat $O/host.json && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_graph_step.py tests/test_gpu_plugins.py -x -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.txt 2>&1 && \
tail -1 $O/pytest.txt && \
timeout -k 10 300 python -u scripts/bench_hccf.py --reps 50 \
    --variants hgd_graph_kernel_adam,hgd_graph_cpu_mask,hgd_graph > $O/hccf.jsonl 2> $O/hccf.err && \
cat $O/hccf.jsonl
