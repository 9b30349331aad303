set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-tune3}
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests/test_gpu_spmm.py tests/test_gpu_ops.py -q -x > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 600 python scripts/tune_spmm.py --rounds 5 --unrolls 8,16 --policies 0,8 > $OUT/uniform.txt 2>&1 || { tail -20 $OUT/uniform.txt; exit 1; }
cat $OUT/uniform.txt
timeout -k 10 600 python scripts/tune_spmm.py --rounds 3 --zipf 1.0 --unrolls 8,16 --policies 0,8 > $OUT/zipf.txt 2>&1 || { tail -20 $OUT/zipf.txt; exit 1; }
cat $OUT/zipf.txt
