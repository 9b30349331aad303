#!/bin/bash
# Round 4: the HCCF eager step on the reference's CPU mask stream with a chain of masks drawn
# ahead (HGD_KEEP_MASK_AHEAD, default 3) at 4 / 8 draw threads, against the device mask and the
# graph variants on the same box. Records under gpurun_out/r04_batch/<tag>.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04_batch/${1:-hccf_rng3}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python -u -m pytest tests/test_sampler.py -x -q > $O/pytest.txt 2>&1 && \
tail -1 $O/pytest.txt && \
for rep in 1 2; do
  for t in 4 8; do
    HGD_EAGER_RNG_THREADS=$t timeout -k 10 200 python -u scripts/bench_hccf.py \
        --variants hgd_cpu_mask,hgd_device_mask > $O/eager_t${t}_r$rep.jsonl 2>&1 || exit 1
  done
done && \
timeout -k 10 200 python -u scripts/bench_hccf.py --variants hgd_graph,hgd_graph_cpu_mask \
    > $O/graph.jsonl 2>&1
rc=$?
for f in $O/*.jsonl; do echo "$f"; grep -h variant $f; done
echo "rc=$rc"
exit $rc
