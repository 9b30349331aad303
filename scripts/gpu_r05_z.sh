#!/bin/bash
# round 5, run z: host profile of the replayed step and the plugin epoch after the padded draw
set -o pipefail
O=gpurun_out/r05/z
mkdir -p $O
timeout -k 10 240 python -u scripts/profile_graph_step_host.py > $O/host.json 2> $O/host.err && \
timeout -k 10 300 python -u scripts/profile_plugin_epoch_host.py > $O/epoch_host.json 2> $O/epoch_host.err && \
timeout -k 10 400 python -u scripts/bench_plugin_epoch.py > $O/plugin_epoch.json 2> $O/plugin_epoch.err
