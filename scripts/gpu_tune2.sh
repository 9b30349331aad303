set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-tune2}
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests/test_gpu_spmm.py -q -x > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 600 python scripts/tune_spmm.py --rounds 5 --unrolls 8,16 --policies 0 > $OUT/uniform.txt 2>&1 || { tail -20 $OUT/uniform.txt; exit 1; }
cat $OUT/uniform.txt
timeout -k 10 600 python scripts/tune_spmm.py --rounds 3 --zipf 1.0 --unrolls 8,16 --policies 0 > $OUT/zipf.txt 2>&1 || { tail -20 $OUT/zipf.txt; exit 1; }
cat $OUT/zipf.txt
for s in 0 1; do HGD_SEGMENTED=$s timeout -k 10 300 python bench.py --pmc off --no-cpu-baseline --steps 20 --warmup 3 > $OUT/bench_seg$s.json 2>/dev/null || exit 1; python -c "import json; b=json.loads(open('$OUT/bench_seg$s.json').read().splitlines()[-1]); print('seg=$s', b['value'], b['ms_per_step'], {k:v['ms'] for k,v in b['roofline']['per_hop'].items()})"; done
