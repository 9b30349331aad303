#!/bin/bash
# Round 4: the HCCF step on the reference's CPU drop-edge stream (HCCF.py:223) on one MI355X —
# eager with the one-mask-ahead prefetch at 4 / 8 / 12 draw threads (HGD_EAGER_RNG_THREADS), and
# replayed from a HIP graph with the next step's masks drawn during the replay; the device-mask
# variants beside them. Records under gpurun_out/r04_batch/<tag>.
#   gpurun --timeout 900 -- 'bash scripts/gpu_r04_hccf_rng.sh <tag>'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04_batch/${1:-hccf_rng}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph_step.py tests/test_sampler.py -x -q \
    --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 && tail -1 $O/pytest.txt && \
timeout -k 10 300 python -u scripts/bench_hccf.py \
    --variants hgd_cpu_mask,hgd_device_mask,hgd_graph,hgd_graph_cpu_mask > $O/hccf.jsonl 2>&1 && \
for t in 4 12; do
  HGD_EAGER_RNG_THREADS=$t timeout -k 10 200 python -u scripts/bench_hccf.py \
      --variants hgd_cpu_mask > $O/hccf_eager_t$t.jsonl 2>&1 || exit 1
done
rc=$?
grep -h variant $O/hccf*.jsonl
echo "rc=$rc"
exit $rc
