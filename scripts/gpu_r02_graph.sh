#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r02_graph
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_graph_step.py tests/test_gpu_infonce.py tests/test_gpu_structure.py -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -50 $OUT/tests.log; exit 1; }
grep -E "PASS|FAIL" $OUT/tests.log | tail -30
timeout -k 10 600 python -u -m pytest tests/test_gpu_plugins.py -x -q --timeout 300 --timeout-method thread -k "execute_end_to_end and (extra6 or extra7)" > $OUT/plugins.log 2>&1 || { tail -50 $OUT/plugins.log; exit 1; }
tail -2 $OUT/plugins.log
timeout -k 10 300 python scripts/bench_hccf.py --variants hgd_device_mask,hgd_graph > $OUT/hccf.json 2> $OUT/hccf.err || { tail -30 $OUT/hccf.err; exit 1; }
cat $OUT/hccf.json
echo ALL_OK
