#!/bin/bash
# HCCF_diffusion iteration on one MI355X: optional GPU tests, scripts/bench_hccf_diffusion.py,
# and a rocprof kernel-trace pass over the step.
# usage: gpu_hccf_diffusion.sh <tag> [pytest args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
O=gpurun_out/$tag
mkdir -p $O
export TMPDIR=/tmp
if [ $# -gt 0 ]; then
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider "$@" \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
fi
timeout -k 10 300 python scripts/bench_hccf_diffusion.py ${HD_VARIANTS:+--variants $HD_VARIANTS} > $O/bench.jsonl 2>&1 \
  || { tail -20 $O/bench.jsonl; exit 1; }
grep variant $O/bench.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python scripts/bench_hccf_diffusion.py --variants ${HD_PROF_VARIANT:-hgd_device_mask} --reps 10 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
find $O/prof -name '*kernel_trace.csv' -exec cp {} $O/kernel_trace.csv \;
rm -rf $O/prof
