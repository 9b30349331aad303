#!/bin/bash
# Round 4: draw-thread sweep for the HCCF step on the reference's CPU mask stream (one MI355X):
# eager one-mask-ahead prefetch at 2 / 3 / 4 / 6 threads, graph replay with the next step's masks
# drawn at 8 / 16 threads. Records under gpurun_out/r04_batch/<tag>.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04_batch/${1:-hccf_rng2}
mkdir -p $O
export TMPDIR=/tmp
for t in 2 3 4 6; do
  HGD_EAGER_RNG_THREADS=$t timeout -k 10 200 python -u scripts/bench_hccf.py \
      --variants hgd_cpu_mask,hgd_device_mask > $O/eager_t$t.jsonl 2>&1 || exit 1
done
for t in 8 16; do
  HGD_CPU_RNG_THREADS=$t timeout -k 10 200 python -u scripts/bench_hccf.py \
      --variants hgd_graph,hgd_graph_cpu_mask > $O/graph_t$t.jsonl 2>&1 || exit 1
done
for f in $O/*.jsonl; do echo "$f"; grep -h variant $f; done
