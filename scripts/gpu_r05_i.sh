#!/bin/bash
# Round 5: the mask staging (next step's masks H2D from the draw worker on a side stream):
# graph-step / plugin tests, then the HCCF step variants and the plugin epoch.
#   gpurun --timeout 900 -- 'bash scripts/gpu_r05_i.sh <tag>'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/${1:-i}
mkdir -p $O
export TMPDIR=/tmp
( while sleep 45; do echo "[r05 i] $(date +%T) $(ls -t $O | head -1)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_graph_step.py tests/test_gpu_plugins.py -x -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.txt 2>&1 && \
tail -1 $O/pytest.txt && \
timeout -k 10 300 python -u scripts/bench_hccf.py --reps 50 \
    --variants hgd_graph_ref_adam,hgd_graph_cpu_mask,hgd_cs_eager_cpu_mask,hgd_graph > $O/hccf.jsonl 2> $O/hccf.err && \
cat $O/hccf.jsonl && \
timeout -k 10 300 python -u scripts/bench_plugin_epoch.py > $O/plugin_epoch.json 2> $O/plugin_epoch.err && \
tail -c 700 $O/plugin_epoch.json
