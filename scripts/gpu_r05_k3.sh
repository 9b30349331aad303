#!/bin/bash
# Round 5: the HCCF step variants incl. the reference's Adam as one captured kernel, then the
# N = 2 / 8 default-flag bench rehearsals. gpurun --timeout 1200 -- 'bash scripts/gpu_r05_k3.sh <tag>'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/${1:-k3}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/bench_hccf.py --reps 50 \
    --variants hgd_graph_kernel_adam,hgd_graph_ref_adam,hgd_graph_cpu_mask,hgd_cs_eager_cpu_mask > $O/hccf.jsonl 2> $O/hccf.err && \
cat $O/hccf.jsonl && \
timeout -k 10 300 python -u scripts/bench_plugin_epoch.py > $O/plugin_epoch.json 2> $O/plugin_epoch.err && \
tail -c 600 $O/plugin_epoch.json || exit 1
REH_N="2 8" bash scripts/gpu_r05_d.sh ${1:-k3}
