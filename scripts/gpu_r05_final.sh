#!/bin/bash
# Round-5 round-end evidence on one MI355X (records under gpurun_out/r05_final/<tag>):
#   gpurun --timeout 1200 -- 'bash scripts/gpu_r05_final.sh <tag> [core|carriers|all]'
#   1. the whole GPU suite (pytest -m gpu) and smoke();
#   2. the default bench line (PMC passes in child processes, CPU baseline on the same graph);
#   3. rocprofv3 --kernel-trace --stats of the bench (no PMC, no CPU baseline);
#   4. the carrier steps (HCCF variants incl. the reference's mask stream and the plugins'
#      graph-replay default with the reference's Adam), the plugin epoch, the skewed-catalogue
#      hop, LocalAware.
# "core" runs 1-3, "carriers" runs 4, "all" (default) both.
# Each step has its own limit; the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05_final/${1:-final}
mkdir -p $O
export TMPDIR=/tmp
( while sleep 45; do echo "[r05 final] $(date +%T) $(ls -t $O | head -1)"; done ) &
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
carriers() {
timeout -k 10 300 python -u scripts/bench_hccf.py \
    --variants hgd_cs_eager_cpu_mask,hgd_graph_kernel_adam,hgd_graph_ref_adam,hgd_graph > $O/hccf.jsonl 2>&1 && \
timeout -k 10 400 python -u scripts/bench_plugin_epoch.py > $O/plugin_epoch.json 2> $O/plugin_epoch.err && \
timeout -k 10 240 python -u scripts/bench_skewed_hop.py > $O/skewed_hop.json 2> $O/skewed_hop.err && \
timeout -k 10 300 python -u scripts/bench_local_aware.py > $O/la.jsonl 2>&1 && echo "carriers ok"
}
case $PART in
  core) core ;;
  carriers) carriers ;;
  *) core && carriers ;;
esac
rc=$?
echo "rc=$rc"
exit $rc
