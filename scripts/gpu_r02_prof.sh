#!/bin/bash
# Round 2 headline evidence: ingest parity, N=1 bench (with its own PMC passes), a kernel-trace
# profile of the same command, zipf with PMC traffic, d=256 with PMC traffic.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r02_prof
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ingest.py -x -q --timeout 200 --timeout-method thread > $OUT/ingest_tests.log 2>&1 || { tail -30 $OUT/ingest_tests.log; exit 1; }
tail -2 $OUT/ingest_tests.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --pmc off --no-cpu-baseline --steps 20 --warmup 5 > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
timeout -k 10 600 python bench.py --workload zipf --pmc on --no-cpu-baseline --steps 10 --warmup 3 > $OUT/bench_zipf.json 2> $OUT/bench_zipf.err || { tail -30 $OUT/bench_zipf.err; exit 1; }
cat $OUT/bench_zipf.json
timeout -k 10 600 python bench.py --dim 256 --pmc on --no-cpu-baseline --steps 10 --warmup 3 > $OUT/bench_d256.json 2> $OUT/bench_d256.err || { tail -30 $OUT/bench_d256.err; exit 1; }
cat $OUT/bench_d256.json
find $OUT -name "*stats.csv"
echo ALL_OK
