#!/bin/bash
# ED-HNN block benches (scripts/bench_edhnn.py) + a kernel-trace profile of the Yelp-shaped run.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/edhnn
timeout -k 10 300 python scripts/bench_edhnn.py > gpurun_out/edhnn/yelp.jsonl 2> gpurun_out/edhnn/yelp.err &&
timeout -k 10 400 python scripts/bench_edhnn.py --users 2000000 --items 200000 --edges 20000000 \
    --reps 20 --cpu-reps 1 --tag synthetic_2M_20M > gpurun_out/edhnn/large.jsonl 2> gpurun_out/edhnn/large.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/edhnn/prof -o run -- \
    python3 scripts/bench_edhnn.py --reps 20 --variants gpu_fused > gpurun_out/edhnn/prof.log 2>&1
echo "rc=$?"
cat gpurun_out/edhnn/*.jsonl
