#!/bin/bash
# Kernel-trace profiles of the §8f layer kernels: ED-HNN block (fused variant only), the MFMA
# Linear microbench, the fused InfoNCE bench; plus the ingest bench. Output: gpurun_out/layers/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/layers
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/edhnn -o run -- \
    python3 scripts/bench_edhnn.py --reps 20 --variants gpu_fused > $O/edhnn.jsonl 2> $O/edhnn.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/linear -o run -- \
    python3 scripts/bench_linear.py --reps 20 > $O/linear.jsonl 2> $O/linear.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/infonce -o run -- \
    python3 scripts/bench_infonce.py --reps 20 > $O/infonce.jsonl 2> $O/infonce.err &&
timeout -k 10 600 python3 scripts/bench_ingest.py > $O/ingest.jsonl 2> $O/ingest.err
echo "rc=$?"
