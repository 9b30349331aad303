set -o pipefail
mkdir -p gpurun_out/ds
for w in ml1m yelp amazon; do
  for g in off on; do
    timeout -k 10 200 python bench.py --workload $w --graph $g --pmc off --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/ds/${w}_$g.json 2> gpurun_out/ds/${w}_$g.err || { tail -5 gpurun_out/ds/${w}_$g.err; exit 1; }
  done
done
for f in gpurun_out/ds/*.json; do python -c "
import json,sys;d=json.load(open('$f'));print('$f',d['value'],d['ms_per_step'],d['config'].get('workload'),d['roofline']['frac'])"; done
