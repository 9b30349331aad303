#!/bin/bash
# round 5: two slot banks / two captured steps — graph-step and plugin tests, host profile, epoch
set -o pipefail
O=gpurun_out/r05/bank
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_graph_step.py tests/test_gpu_plugins.py tests/test_gpu_adam.py > $O/pytest.txt 2>&1 && \
timeout -k 10 200 python -u scripts/profile_graph_step_host.py > $O/host.json 2> $O/host.err && \
timeout -k 10 300 python -u scripts/profile_plugin_epoch_host.py > $O/epoch_host.json 2> $O/epoch_host.err
