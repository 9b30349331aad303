set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-tune}; shift || true
mkdir -p $OUT
timeout -k 10 600 python scripts/tune_spmm.py --rounds 5 > $OUT/uniform.txt 2>&1 || { tail -20 $OUT/uniform.txt; exit 1; }
cat $OUT/uniform.txt
timeout -k 10 600 python scripts/tune_spmm.py --rounds 3 --zipf 1.0 > $OUT/zipf.txt 2>&1 || { tail -20 $OUT/zipf.txt; exit 1; }
cat $OUT/zipf.txt
