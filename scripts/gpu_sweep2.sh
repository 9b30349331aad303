set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-sweep2}
mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m gpu -q -x > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
run() {
  name=$1; shift
  timeout -k 10 300 python bench.py --pmc off --no-cpu-baseline --steps 20 --warmup 3 "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "FAIL $name"; tail -5 $OUT/$name.err; return 1; }
  python -c "import json; b=json.loads(open('$OUT/$name.json').read().splitlines()[-1]); r=b['roofline']; print('$name', b['value'], b['ms_per_step'], r['achieved'], r['frac'], {k:v['ms'] for k,v in r.get('per_hop',{}).items()})"
}
run synth && run synth_nograph --graph off && run ml1m --workload ml1m && run ml1m_nograph --workload ml1m --graph off && run yelp --workload yelp && run amazon --workload amazon --dim 128 && run zipf --workload zipf
