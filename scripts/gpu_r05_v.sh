#!/bin/bash
# round 5, run v: adaptive split threshold + BPR heavy rows — full GPU suite, skewed hop, epoch
set -o pipefail
O=gpurun_out/r05/v
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
  > $O/pytest.txt 2>&1 && \
timeout -k 10 240 python -u scripts/bench_skewed_hop.py > $O/skewed_hop.json 2> $O/skewed_hop.err && \
timeout -k 10 300 python -u scripts/profile_plugin_epoch_host.py > $O/epoch_host.json 2> $O/epoch_host.err
