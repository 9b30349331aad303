# A/B full-step bench over tuning env settings, interleaved twice
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab}; shift || true
mkdir -p $OUT
for rep in 1 2; do
for cfg in "8 0" "8 1" "16 0" "16 1"; do
  set -- $cfg
  HGD_SPMM_UNROLL=$1 HGD_SPMM_POLICY=$2 timeout -k 10 300 python bench.py --pmc off --no-cpu-baseline --steps 20 --warmup 3 ${WL:-} > $OUT/b_$1_$2_$rep.json 2>/dev/null || exit 1
  python -c "import json,sys; b=json.loads(open('$OUT/b_$1_$2_$rep.json').read().splitlines()[-1]); print('U=$1 P=$2', b['value'], b['ms_per_step'], {k:v['ms'] for k,v in b['roofline']['per_hop'].items()})"
done
done
