#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r02_sharded
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_sharded_encoders.py tests/test_gpu_config_parity.py tests/test_gpu_plugins.py -x -q --timeout 400 --timeout-method thread -k "sharded" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
for m in local_aware hccf; do
timeout -k 10 300 python scripts/bench_sharded_encoder.py --model $m > $OUT/n1_$m.json 2> $OUT/n1_$m.err || { tail -20 $OUT/n1_$m.err; exit 1; }
cat $OUT/n1_$m.json
done
echo ALL_OK
