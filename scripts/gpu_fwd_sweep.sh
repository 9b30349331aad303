#!/bin/bash
# Forward / backward-data row GEMM at 144,242 x 128 -> 128 over the existing tuning knobs
# (HGD_X3_COLS, HGD_X3S_TILES, HGD_ROWGEMM_BLOCKS), defaults first and last. One MI355X.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/fwdsweep; mkdir -p $O; export TMPDIR=/tmp
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 60 python scripts/bench_linear.py --rows 144242 --dim 128 --cases fwd_hgd bwd_data_hgd > $O/$lab.jsonl 2>&1 || { cat $O/$lab.jsonl; exit 1; }
  echo "$lab $(grep -ho '"case": "[a-z_]*".*"us": [0-9.]*' $O/$lab.jsonl | sed 's/"rows.*"us"/us/' | tr '\n' ' ')"
}
run default0 HGD_X3_COLS=0
run cols64 HGD_X3_COLS=64
run cols128 HGD_X3_COLS=128
run tiles1 HGD_X3S_TILES=1
run tiles2 HGD_X3S_TILES=2
run tiles3 HGD_X3S_TILES=3
for b in 256 384 768 1024; do run blocks$b HGD_ROWGEMM_BLOCKS=$b; done
run default1 HGD_X3_COLS=0
