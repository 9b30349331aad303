#!/bin/bash
# Kernel trace + PMC passes of the skinny-product kernels at the Amazon d = 128 shape (VERDICT r2
# next 3: traffic ÷ algorithmic and where the time goes). One counter group per pass.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/proflin
mkdir -p $O
export TMPDIR=/tmp
CMD="python scripts/bench_linear.py --rows 144242 --dim 128 --reps 5 --inner 4 --cases fwd_hgd bwd_data_hgd bwd_weight_hgd fwd_drop_res_hgd"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- $CMD > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
n=0
for pmc in "FETCH_SIZE WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" "SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC" "SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY"; do
  n=$((n+1))
  timeout -s KILL 90 rocprofv3 --pmc $pmc -d $O/pmc$n -o run -- $CMD > $O/pmc$n.log 2>&1 || { echo "pmc pass $n failed"; tail -5 $O/pmc$n.log; }
done
find $O -name "*.csv" | head -20
