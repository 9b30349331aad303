# Profile the default bench workload: kernel trace + stats (CSV), then separate PMC passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-prof}
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -m gpu -q -x > $OUT/tests.log 2>&1 || { echo TESTFAIL; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 900 python bench.py --steps 20 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { echo BENCHFAIL; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python bench.py --pmc off --no-cpu-baseline --steps 20 --warmup 3 > $OUT/trace.log 2>&1 || { echo PROFFAIL; tail -20 $OUT/trace.log; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$c -o run -- python bench.py --pmc off --no-cpu-baseline --steps 3 --warmup 1 > $OUT/pmc_$c.log 2>&1 || { echo PMCFAIL $c; tail -20 $OUT/pmc_$c.log; exit 1; }
done
timeout -k 10 600 python bench.py --workload zipf --pmc off --no-cpu-baseline --steps 10 --warmup 2 > $OUT/bench_zipf.json 2>&1 || { echo ZIPFFAIL; tail -30 $OUT/bench_zipf.json; exit 1; }
cat $OUT/bench_zipf.json
find $OUT -name "*.csv" | head -20
