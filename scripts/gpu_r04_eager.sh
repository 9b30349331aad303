#!/bin/bash
# Round 4: HCCF eager-step variants (compacted vs capture-safe drop-edge on the reference's CPU
# mask stream) and the plugin epoch (eager, capture-safe eager, hgd_graph). Records under
# gpurun_out/r04_batch/<tag>:  gpurun --timeout 600 -- 'bash scripts/gpu_r04_eager.sh <tag>'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04_batch/${1:-eager}
mkdir -p $O
export TMPDIR=/tmp
( while sleep 45; do echo "[eager] $(date +%T) $(ls -t $O | head -1)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
V=hgd_cpu_mask,hgd_device_mask,hgd_capture_safe_eager,hgd_cs_eager_cpu_mask,hgd_graph,hgd_graph_cpu_mask
timeout -k 10 300 python -u scripts/bench_hccf.py --reps 50 --variants $V > $O/hccf.jsonl 2>&1 && \
cat $O/hccf.jsonl | grep '^{' && \
timeout -k 10 300 python -u scripts/bench_plugin_epoch.py --ref-steps 10 > $O/epoch.json 2>&1 && \
grep '^{' $O/epoch.json
rc=$?
echo "rc=$rc"
exit $rc
