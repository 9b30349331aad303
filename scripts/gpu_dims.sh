# headline bench at the other BASELINE widths (d = 128 Amazon-Book, d = 256 configs[4]) + d = 32
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-dims}
mkdir -p $OUT
for d in 256 128 32; do
  timeout -k 10 300 python bench.py --pmc off --no-cpu-baseline --steps 5 --warmup 2 --dim $d > $OUT/d$d.json 2> $OUT/d$d.err || { tail -20 $OUT/d$d.err; exit 1; }
  python -c "import json;b=json.loads(open('$OUT/d$d.json').read().strip().splitlines()[-1]);r=b['roofline'];print($d, b['value'], b['ms_per_step'], r['achieved'], r['frac'], r.get('per_hop'))"
done
