#!/bin/bash
# rocprof kernel stats of the small-shape dense kernels (scripts/bench_small_kernels.py).
# usage: gpu_small.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-small}
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp
cd /tmp
for case in hgnn linear infonce; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/$tag/prof_$case" -o run -- \
    python3 "$GRAFT_REPO_ROOT/scripts/bench_small_kernels.py" --cases $case >> "$GRAFT_REPO_ROOT/gpurun_out/$tag/bench.jsonl" 2> "$GRAFT_REPO_ROOT/gpurun_out/$tag/err_$case.log" || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/$tag/err_$case.log"; exit 1; }
done
cd "$GRAFT_REPO_ROOT"
cat gpurun_out/$tag/bench.jsonl
for case in hgnn linear infonce; do
  f=$(find gpurun_out/$tag/prof_$case -name '*kernel_stats.csv' | head -1)
  cp "$f" gpurun_out/$tag/kernel_stats_$case.csv
  echo "== $case"
  python3 - "gpurun_out/$tag/kernel_stats_$case.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print(f"{int(r['Calls']):6d} {float(r['AverageNs'])/1000:8.2f}us {r['Name'][:110]}")
PY
done
