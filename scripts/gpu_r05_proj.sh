#!/bin/bash
# round 5: grouped table projections — HCCF tests, config parity, step time, epoch
set -o pipefail
O=gpurun_out/r05/proj
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_hccf_layers.py tests/test_gpu_graph_step.py tests/test_gpu_plugins.py \
  tests/test_gpu_config_parity.py > $O/pytest.txt 2>&1 && \
timeout -k 10 300 python -u scripts/bench_hccf.py \
    --variants hgd_graph_kernel_adam,hgd_cs_eager_cpu_mask,hgd_graph > $O/hccf.jsonl 2>&1 && \
timeout -k 10 300 python -u scripts/profile_plugin_epoch_host.py > $O/epoch_host.json 2> $O/epoch_host.err
