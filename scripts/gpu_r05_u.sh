#!/bin/bash
# round 5, run u: BPR heavy-row kernel, skewed hop split plans, Zipf epoch profile
set -o pipefail
O=gpurun_out/r05/u
mkdir -p $O
P=$GRAFT_REPO_ROOT/$O/prof
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_hccf_layers.py tests/test_gpu_plugins.py > $O/pytest.txt 2>&1 && \
timeout -k 10 240 python -u scripts/bench_skewed_hop.py > $O/skewed_hop.json 2> $O/skewed_hop.err && \
timeout -k 10 300 python -u scripts/profile_plugin_epoch_host.py > $O/epoch_host.json 2> $O/epoch_host.err && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $P -o epoch -- python3 scripts/profile_plugin_epoch_host.py > $O/epoch_host_prof.json 2> $O/prof.log; rc=$?
find $P -name "*kernel_trace.csv" -delete 2>/dev/null
exit $rc
