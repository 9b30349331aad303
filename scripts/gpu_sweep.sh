# bench sweep over widths and workloads (one line each)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-sweep}
mkdir -p $OUT
run() {
  name=$1; shift
  timeout -k 10 300 python bench.py --pmc off --no-cpu-baseline --steps 10 --warmup 2 "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "FAIL $name"; tail -5 $OUT/$name.err; return 1; }
  python -c "import json; b=json.loads(open('$OUT/$name.json').read().splitlines()[-1]); r=b['roofline']; print('$name', b['value'], b['ms_per_step'], r['achieved'], r['frac'], {k:v['ms'] for k,v in r.get('per_hop',{}).items()})"
}
run d32 --dim 32 && run d128 --dim 128 && run d256 --dim 256 --edges 50000000 --users 5000000 && run ml1m --workload ml1m && run yelp --workload yelp && run amazon --workload amazon --dim 128 && run zipf_d128 --workload zipf --dim 128
