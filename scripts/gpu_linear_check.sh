#!/bin/bash
# Row-GEMM change check on one MI355X: the linear / fused-dropout / encoder / config-parity GPU
# tests, the linear microbench at the carriers' shapes and the LocalAware / HCCF steps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/lincheck
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_linear.py tests/test_gpu_fused_dropout.py tests/test_gpu_encoders.py tests/test_gpu_config_parity.py tests/test_gpu_hccf_layers.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python scripts/bench_linear.py --rows 69716 31668 > $O/lin64.jsonl 2>&1 || { cat $O/lin64.jsonl; exit 1; }
timeout -k 10 120 python scripts/bench_linear.py --rows 144242 --dim 128 > $O/lin128.jsonl 2>&1 || { cat $O/lin128.jsonl; exit 1; }
grep -h hgd $O/lin64.jsonl $O/lin128.jsonl
timeout -k 10 200 python scripts/bench_local_aware.py > $O/la.jsonl 2>&1 || { tail $O/la.jsonl; exit 1; }
grep -h ms $O/la.jsonl
timeout -k 10 300 python scripts/bench_hccf.py --variants hgd_graph > $O/hccf.jsonl 2>&1 || { tail $O/hccf.jsonl; exit 1; }
grep -h variant $O/hccf.jsonl
