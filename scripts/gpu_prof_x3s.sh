#!/bin/bash
# PMC passes of the dense products at 144,242 × 128 → 128 (one counter group per pass), for each
# HGD_X3S_TILES setting in PROF_TILES (0 = default) and the bench_linear cases in PROF_CASES.
# FETCH_SIZE on gfx950 reports half the bytes of 16-B-per-lane streaming reads (MI355X_MICROARCH
# § HBM): double it before comparing. Records under gpurun_out/profx3s/.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/profx3s
mkdir -p $O
export TMPDIR=/tmp
CASES=${PROF_CASES:-fwd_hgd}
CMD="python scripts/bench_linear.py --rows 144242 --dim 128 --reps 5 --inner 4 --cases $CASES"
for t in ${PROF_TILES:-0}; do
  n=0
  for pmc in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
      "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
      "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM SQ_VALU_MFMA_BUSY_CYCLES" \
      "FETCH_SIZE" "WRITE_SIZE"; do
    n=$((n+1))
    HGD_X3S_TILES=$t timeout -s KILL 90 rocprofv3 --pmc $pmc --output-format csv -d $O/t${t}_pmc$n -o run -- $CMD \
      > $O/t${t}_pmc$n.log 2>&1 || { echo "pmc pass $n failed"; tail -5 $O/t${t}_pmc$n.log; exit 1; }
  done
done
python3 - $O <<'PY'
import csv, glob, collections, sys, os, re
O = sys.argv[1]
# per kernel (template arguments kept), per counter: mean over dispatches of the per-dispatch sum
for d in sorted(glob.glob(os.path.join(O, "t*_pmc*"))):
    for f in glob.glob(os.path.join(d, "run_counter_collection.csv")):
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "k_row_gemm" not in k and "k_splitk" not in k:
                continue
            k = re.sub(r"\(.*$", "", k.replace("hgd::", "").replace("lin::", "").replace("(anonymous namespace)::", ""))
            per[(k, r["Counter_Name"])][r["Dispatch_Id"]] += float(r["Counter_Value"])
        for (k, c), v in sorted(per.items()):
            print(os.path.basename(d), k, c, round(sum(v.values()) / len(v)))
PY
