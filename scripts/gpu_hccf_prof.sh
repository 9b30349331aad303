# HCCF training step: bench (all variants) + kernel trace of the device-mask variant
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-hccf}
mkdir -p $O
timeout -k 10 300 python3 scripts/bench_hccf.py > $O/bench.jsonl 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 scripts/bench_hccf.py --variants hgd_device_mask > $O/trace.jsonl 2> $O/trace.err || { tail -20 $O/trace.err; exit 1; }
find $O/trace -name "*kernel_stats.csv"
