#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r02_graph_prof
mkdir -p $OUT
timeout -k 10 300 python scripts/bench_hccf.py --variants hgd_capture_safe_eager,hgd_graph > $OUT/hccf.json 2> $OUT/hccf.err || { tail -30 $OUT/hccf.err; exit 1; }
cat $OUT/hccf.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 scripts/bench_hccf.py --variants hgd_graph --reps 5 > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
echo ALL_OK
