#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r02_linear
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_linear.py tests/test_gpu_layers.py tests/test_gpu_config_parity.py -x -q --timeout 400 --timeout-method thread -k "not sharded" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python scripts/bench_linear.py --rows 31668 69716 144242 2200000 > $OUT/linear.jsonl 2>&1 || { tail -20 $OUT/linear.jsonl; exit 1; }
cat $OUT/linear.jsonl
timeout -k 10 300 python scripts/bench_linear.py --rows 144242 --dim 128 >> $OUT/linear.jsonl 2>&1 || exit 1
timeout -k 10 300 python scripts/bench_hccf.py --variants hgd_device_mask > $OUT/hccf.json 2>&1 || { tail -20 $OUT/hccf.json; exit 1; }
cat $OUT/hccf.json
echo ALL_OK
