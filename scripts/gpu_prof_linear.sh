#!/bin/bash
# Kernel trace + PMC passes of the skinny-product kernels at the Amazon d = 128 shape (VERDICT r2
# next 3: traffic ÷ algorithmic and where the time goes). One counter group per pass; FETCH_SIZE
# (3 TCC slots) and WRITE_SIZE (2) each take a pass of their own. PROF_CASES picks the cases.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/proflin
mkdir -p $O
export TMPDIR=/tmp
CASES=${PROF_CASES:-"fwd_hgd bwd_data_hgd bwd_weight_hgd fwd_drop_res_hgd"}
CMD="python scripts/bench_linear.py --rows 144242 --dim 128 --reps 5 --inner 4 --cases $CASES"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $CMD \
  > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
n=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" \
    "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
    "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
    "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM SQ_VALU_MFMA_BUSY_CYCLES"; do
  n=$((n+1))
  timeout -s KILL 90 rocprofv3 --pmc $pmc --output-format csv -d $O/pmc$n -o run -- $CMD \
    > $O/pmc$n.log 2>&1 || { echo "pmc pass $n failed"; tail -5 $O/pmc$n.log; exit 1; }
done
find $O -name "*.csv" | head -20
