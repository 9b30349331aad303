# tests + one bench line (+ optional extra bench args)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-quick}; shift || true
mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m gpu -q > $OUT/tests.log 2>&1; rc=$?
tail -15 $OUT/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python bench.py --pmc off --no-cpu-baseline --steps 10 --warmup 2 "$@" > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
