# per-variant kernel stats of one ED-HNN block (Yelp-shaped), summaries only
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for form in ${FORMS:-mean spmm}; do
  for fused in 1 0; do
    d=gpurun_out/prof_edhnn_${form}_${fused}
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 scripts/dev/edhnn_one.py --form $form --fused $fused --steps 100 > $d.log 2>&1
    find $d -name "*kernel_trace.csv" -delete
  done
done
