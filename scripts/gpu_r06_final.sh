#!/bin/bash
# Round-6 evidence on one MI355X (records under gpurun_out/r06_round/<tag>):
#   gpurun --timeout 1200 -- 'bash scripts/gpu_r06_final.sh <tag> [core|coreskew|d256|d256zipf|skewed|zipf|all]'
#   core:   the whole GPU suite (pytest -m gpu), smoke(), the default bench line (PMC passes in
#           child processes, CPU baseline + parity gate on the same graph), rocprofv3
#           --kernel-trace --stats of the bench;
#   d256:   the same bench line at configs[4]'s width (--dim 256) and its rocprof pass;
#   skewed: the skewed-catalogue teacher-forced plugin test (1e-5 outright) with its record (-s),
#   zipf:   the Yelp-shaped Zipf teacher-forced record with the reference's fp32 calls
#           re-run in other entry orders where ours exceeds their deviation.
# Each step has its own limit; the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06_round/${1:-final}
mkdir -p $O
export TMPDIR=/tmp
( while sleep 45; do echo "[r06 final] $(date +%T) $(ls -t $O | head -1)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
git_head=$(cat .git_head 2>/dev/null || echo unknown)
echo "HEAD $git_head" > $O/HEAD.txt
PART=${2:-all}
core() {
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $O/pytest.txt 2>&1 && tail -1 $O/pytest.txt && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 && \
tail -1 $O/smoke.txt && \
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err && echo "bench ok" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python bench.py --no-cpu-baseline --pmc off > $O/bench_prof.json 2> $O/bench_prof.err && \
find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/bench_kernel_stats.csv \; && \
rm -rf $O/prof && echo "prof ok"
}
d256() {
timeout -k 10 900 python -u bench.py --dim 256 > $O/bench_d256.json 2> $O/bench_d256.err && \
echo "bench d256 ok" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof256 -o run -- \
    python bench.py --dim 256 --no-cpu-baseline --pmc off > $O/bench_d256_prof.json \
    2> $O/bench_d256_prof.err && \
find $O/prof256 -name '*kernel_stats.csv' -exec cp {} $O/bench_d256_kernel_stats.csv \; && \
rm -rf $O/prof256 && echo "prof d256 ok"
}
skewed() {
timeout -k 10 400 python -u -m pytest -s -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider -m gpu \
    "tests/test_gpu_plugins.py::test_hccf_skewed_catalogue_steps_match_reference_ops" \
    > $O/bounds_skewed.txt 2>&1 && grep "skewed-catalogue record" $O/bounds_skewed.txt
}
zipf() {
timeout -k 10 900 python -u scripts/diag/diag_zipf_teacher_forced.py --start 150 --stop 290 \
    --orders 3 --analyze 0 > $O/zipf_orders.jsonl 2> $O/zipf_orders.err && tail -1 $O/zipf_orders.jsonl
}
case $PART in
  core) core ;;
  coreskew) core && skewed ;;
  d256) d256 ;;
  d256zipf) d256 && zipf ;;
  skewed) skewed ;;
  zipf) zipf ;;
  *) core && d256 && skewed && zipf ;;
esac
rc=$?
echo "rc=$rc"
exit $rc
