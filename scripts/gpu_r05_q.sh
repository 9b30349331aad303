#!/bin/bash
# round 5, run q: device sampler staging, deferred loss reads (run-ahead), chunked MT jump
set -o pipefail
O=gpurun_out/r05/q
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_sampler_device.py tests/test_gpu_graph_step.py tests/test_gpu_plugins.py \
  > $O/pytest.txt 2>&1 && \
timeout -k 10 240 python -u scripts/profile_graph_step_host.py > $O/host.json 2> $O/host.err && \
timeout -k 10 400 python -u scripts/bench_plugin_epoch.py > $O/plugin_epoch.json 2> $O/plugin_epoch.err
