set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/t2.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/t2.log; }
timeout -k 10 600 python bench.py --pmc off --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/b2.log 2>&1 || { echo BENCHFAIL; tail -30 gpurun_out/b2.log; exit 1; }
cat gpurun_out/b2.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2 -o run -- python bench.py --pmc off --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/p2.log 2>&1 || { echo PROFFAIL; tail -20 gpurun_out/p2.log; }
find gpurun_out/prof2 -name "*stats*"
