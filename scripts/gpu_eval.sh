# top-K evaluation: parity tests, bench, kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-eval}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_topk.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 scripts/bench_eval.py > $O/bench.jsonl 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 scripts/bench_eval.py --cpu-sample 1 > $O/trace.jsonl 2> $O/trace.err || { tail -20 $O/trace.err; exit 1; }
head -8 $(find $O/trace -name "*kernel_stats.csv")
