#!/bin/bash
# Round 5: the mask stager waits on its worker thread for the bank's last reader before the
# host → device copy. GPU tests of the replayed step / plugins, then the carrier timings.
#   gpurun --timeout 900 -- 'bash scripts/gpu_r05_hostwait.sh <tag>'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/${1:-hostwait}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_graph_step.py tests/test_gpu_plugins.py \
    tests/test_gpu_hccf_layers.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    > $O/pytest.txt 2>&1 && tail -1 $O/pytest.txt && \
timeout -k 10 300 python -u scripts/bench_hccf.py --variants hgd_graph_ref_adam,hgd_graph_kernel_adam \
    > $O/hccf.jsonl 2>&1 && \
timeout -k 10 400 python -u scripts/bench_plugin_epoch.py > $O/plugin_epoch.json 2> $O/plugin_epoch.err && \
echo "hostwait ok"
