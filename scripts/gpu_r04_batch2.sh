#!/bin/bash
# Round-4 batch 2 on one MI355X (records under gpurun_out/r04_batch/<tag>):
#   gpurun --timeout 1500 -- 'bash scripts/gpu_r04_batch2.sh <tag>'
#   1. bench.py --gpus 2 --transport auto --check rehearsal (gloo setup, one device) on a 10 M-edge
#      graph: the transport probe's choice, fallbacks and the sharded check;
#   2. the headline bench line (default flags: PMC passes, the CPU baseline on the same graph);
#   3. rocprofv3 kernel stats of the same bench (no PMC, no CPU baseline);
#   4. the HCCF step with the reference's CPU keep-mask stream at the default RNG threads, eager
#      and replayed from a HIP graph (masks drawn on the host before each replay).
# (first: the graph-step and plugin GPU tests)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04_batch/${1:-run2}
mkdir -p $O
export TMPDIR=/tmp
( while sleep 45; do echo "[r04 batch2] $(date +%T) $(ls -t $O | head -1)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_graph_step.py tests/test_gpu_plugins.py -x -v \
    -rw --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 && echo "pytest ok" && \
HGD_DIST_BACKEND=gloo HGD_STALL_DUMP_S=200 timeout -k 10 300 python -u bench.py --gpus 2 --check \
    --no-cpu-baseline --pmc off --users 1000000 --items 100000 --edges 10000000 --steps 3 \
    --warmup 1 > $O/auto_n2.json 2> $O/auto_n2.err && echo "auto n2 ok" && \
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err && echo "bench ok" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python bench.py --no-cpu-baseline --pmc off > $O/bench_prof.json 2> $O/bench_prof.err && \
find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/bench_kernel_stats.csv \; && \
rm -rf $O/prof && echo "prof ok" && \
timeout -k 10 300 python -u scripts/bench_hccf.py \
    --variants hgd_cpu_mask,hgd_device_mask,hgd_graph,hgd_graph_cpu_mask \
    > $O/hccf.jsonl 2>&1 && echo "hccf ok"
rc=$?
echo "rc=$rc"
exit $rc
