#!/bin/bash
# Row-GEMM change check on one MI355X: the linear GPU tests first, the linear microbench at the
# carriers' shapes for the split-bf16 default and the exact f32-MFMA kernels (HGD_GEMM_EXACT=1),
# then the fused-dropout / encoder / config-parity tests and the LocalAware / HCCF steps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/lincheck
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_linear.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_linear.log 2>&1 || { tail -30 $O/pytest_linear.log; exit 1; }
tail -1 $O/pytest_linear.log
for ex in 0 1; do
  HGD_GEMM_EXACT=$ex timeout -k 10 120 python scripts/bench_linear.py --rows 69716 31668 > $O/lin64_exact$ex.jsonl 2>&1 || { cat $O/lin64_exact$ex.jsonl; exit 1; }
  HGD_GEMM_EXACT=$ex timeout -k 10 120 python scripts/bench_linear.py --rows 144242 --dim 128 > $O/lin128_exact$ex.jsonl 2>&1 || { cat $O/lin128_exact$ex.jsonl; exit 1; }
  echo "== HGD_GEMM_EXACT=$ex"
  grep -h hgd $O/lin64_exact$ex.jsonl $O/lin128_exact$ex.jsonl
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python scripts/bench_local_aware.py > $O/la.jsonl 2>&1 || { tail $O/la.jsonl; exit 1; }
grep -h ms $O/la.jsonl
timeout -k 10 300 python scripts/bench_hccf.py --variants hgd_graph > $O/hccf.jsonl 2>&1 || { tail $O/hccf.jsonl; exit 1; }
grep -h variant $O/hccf.jsonl
